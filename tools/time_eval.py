"""A/B of the evaluate() scope (hh_decode_host: host payload in, host
symbols out, chunk pipeline) on the 1 GiB kjv-tiled stream, for the library
named by HIPHUFF_LIB; one JSON line (median and min of N calls).
    python tools/time_eval.py [MiB] [reps]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
cache = os.environ.get("HH_TEXT_CACHE")
if cache and os.path.exists(cache):
    hf = H.HuffFile.load(os.path.join(ROOT, "files", "kjv.txt.huff"))
    text = np.load(cache)
else:
    hf, text = synth.load_source(os.path.join(ROOT, "files"), "kjv.txt")
syn = synth.tiled_stream(hf, text, mib << 20)
host = syn.data[: syn.compressed_bytes].cpu().numpy()
n = syn.decoded_bytes
dec = H.Decoder(0)
dec.set_tree(syn.tree)
buf = np.zeros(n + 16, np.uint8)
out = dec.decode_host(host, syn.bits, n + 16, out=buf)
ok = len(out) == n and synth.verify_tiled(torch.from_numpy(out).cuda(), syn)
ts = []
for _ in range(reps):
    buf[:] = 0
    t0 = time.perf_counter()
    dec.decode_host(host, syn.bits, n + 16, out=buf)
    ts.append(time.perf_counter() - t0)
print(json.dumps({"lib": os.path.basename(os.environ.get("HIPHUFF_LIB", H.LIB_PATH)), "mib": mib, "ok": bool(ok),
                  "ms": round(statistics.median(ts) * 1e3, 2), "ms_min": round(min(ts) * 1e3, 2),
                  "chunk_kb": os.environ.get("HH_PIPE_CHUNK_KB")}))
