"""Size sweep of the device-resident decode (north_star: 64 MiB .. 8 GiB per
GPU): the kjv-tiled stream at each compressed size, decoded RUNS times on one
GPU; median device time of the pipeline (the decoder's HIP events), decoded
MB/s and the HBM roofline fraction of (C + D) algorithmic bytes.  Every size
is checked against the tiled text first.  Writes one JSON document.

    python tools/sweep.py OUT.json [MiB ...]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0
out_path = sys.argv[1]
sizes = [int(x) for x in sys.argv[2:]] or [64, 128, 256, 512, 1024, 2048, 4096, 8192]
runs = int(os.environ.get("RUNS", "5"))
hf, text = synth.load_source(os.path.join(ROOT, "files"), "kjv.txt")
rows = []
for mib in sizes:
    t0 = time.time()
    syn = synth.tiled_stream(hf, text, mib << 20)
    dec = H.Decoder(0)
    dec.set_tree(syn.tree)
    out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
    n = dec.decode_device(syn.data, syn.bits, out)
    torch.cuda.synchronize()
    ok = n == syn.decoded_bytes and synth.verify_tiled(out, syn)
    ms = []
    for _ in range(runs):
        dec.decode_device(syn.data, syn.bits, out)
        ms.append(dec.stats())
    torch.cuda.synchronize()
    # wall time per decode in a stream of asynchronous decodes (as bench.py)
    lens = []
    t1 = time.perf_counter()
    for _ in range(runs * 4):
        lens.append(dec.decode_device_async(syn.data, syn.bits, out))
    dec.wait()
    torch.cuda.synchronize()
    ms_step = (time.perf_counter() - t1) / (runs * 4) * 1e3
    ok = ok and all(int(x.value) == syn.decoded_bytes for x in lens)
    t = statistics.median(s["ms_total"] for s in ms)
    C, D = syn.compressed_bytes, syn.decoded_bytes
    row = {"MiB": mib, "bits": syn.bits, "decoded_bytes": D, "ok": bool(ok),
           "ms_total": round(t, 4),
           "decoded_MBps": round(D / (t * 1e-3) / 1e6, 1),
           "ms_step_async": round(ms_step, 4), "decoded_MBps_wall": round(D / (ms_step * 1e-3) / 1e6, 1),
           "roofline_frac": round((C + D) / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "fast_path": all(s["exact_fallback"] == 0 for s in ms)}
    rows.append(row)
    print(json.dumps(row), f"({time.time() - t0:.1f} s)", flush=True)
    dec.close()
    del out, syn
    torch.cuda.empty_cache()
doc = {"workload": "synthetic kjv-tiled .huff (files/kjv.txt.huff codebook), device-resident",
       "runs": runs, "gpu": torch.cuda.get_device_name(0), "rows": rows}
with open(out_path, "w") as f:
    json.dump(doc, f, indent=1)
