"""Small streams: the single pass (k_one, HH_ONE=1) against the two passes,
device time per decode (the decoder's HIP events, median of N runs) on the
kjv-tiled stream from 256 KiB to 64 MiB, every output verified.

    python tools/small_one_vs_two.py [runs]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 21
hf, text = synth.load_source(os.path.join(ROOT, "files"), "kjv.txt")
for kib in (256, 1024, 4096, 16384, 65536):
    syn = synth.tiled_stream(hf, text, kib << 10)
    out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
    row = {"KiB": kib, "tiles": None}
    for name, one in (("two", "0"), ("one", "1")):
        os.environ["HH_ONE"] = one
        dec = H.Decoder(0)
        dec.set_tree(syn.tree)
        row["tiles"] = (syn.bits + dec.tile_bits() - 1) // dec.tile_bits()
        ms, ok, sm = [], True, None
        for _ in range(runs):
            n = dec.decode_device(syn.data, syn.bits, out)
            torch.cuda.synchronize()
            st = dec.stats()
            ms.append(st["ms_total"])
            sm = st["state_machine"]
            ok = ok and n == syn.decoded_bytes
        ok = ok and synth.verify_tiled(out, syn)
        dec.close()
        row[name] = {"ms": round(statistics.median(ms), 4), "ok": bool(ok), "sm": sm}
    print(json.dumps(row), flush=True)
