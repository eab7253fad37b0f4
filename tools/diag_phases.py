"""Diagnostic only: device time of the fused kernel stopped after each phase.

HIPHUFF_DIAG_STOP=k makes the kernel skip everything after phase k
(1 staging, 2 region decode + walks, 3 tile table, 4 look-back, 0 = full);
the decoder reads it when it is created.  Timings are cumulative.
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    stops = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3", "4"]
    os.environ.pop("HIPHUFF_DIAG_STOP", None)
    log("import torch")
    import torch
    import huffmandecoderongpus_amd as H
    from huffmandecoderongpus_amd import synth
    log("load source")
    hf, text = synth.load_source(os.path.join(ROOT, "files"))
    syn = synth.tiled_stream(hf, text, size << 20)
    torch.cuda.synchronize()
    out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
    log(f"stream ready: {syn.bits} bits")
    for stop in stops:
        os.environ["HIPHUFF_DIAG_STOP"] = stop
        dec = H.Decoder(0)
        dec.set_tree(syn.tree)
        ms = []
        for _ in range(5):
            dec.decode_device(syn.data, syn.bits, out)
            ms.append(dec.stats()["ms_total"])
        dec.close()
        log(f"stop={stop} ms={statistics.median(ms[1:]):.4f} all={[round(x, 3) for x in ms]}")


if __name__ == "__main__":
    main()
