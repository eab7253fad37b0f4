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
aff = os.environ.get("HH_EVAL_AFFINITY")   # local | remote: the host buffers first touched on the GPU's NUMA node or the other
cpus = None
if aff:
    import bench
    loc = bench.gpu_local_cpus(0) or set()
    cpus = loc if aff == "local" else (os.sched_getaffinity(0) - loc)
    os.sched_setaffinity(0, cpus)
host = np.array(syn.data[: syn.compressed_bytes].cpu().numpy(), copy=True)
n = syn.decoded_bytes
dec = H.Decoder(0, flags=int(os.environ.get("HH_EVAL_FLAGS", "0")))
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
res = {"lib": os.path.basename(os.environ.get("HIPHUFF_LIB", H.LIB_PATH)), "mib": mib, "ok": bool(ok),
       "flags": os.environ.get("HH_EVAL_FLAGS", "0"),
       "ms": round(statistics.median(ts) * 1e3, 2), "ms_min": round(min(ts) * 1e3, 2),
       "all_ms": [round(t * 1e3, 2) for t in ts], "chunk_kb": os.environ.get("HH_PIPE_CHUNK_KB"),
       "affinity": aff, "cpus": len(cpus) if cpus else None}
if os.environ.get("HH_EVAL_DMA"):
    # the PCIe floor: the same byte counts moved by plain async copies
    # between pinned host tensors and the GPU, each way alone and both at once
    hin = torch.from_numpy(host).pin_memory()
    hout = torch.empty(n, dtype=torch.uint8).pin_memory()
    din = torch.empty(hin.numel(), dtype=torch.uint8, device="cuda")
    dout = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def t(f):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) * 1e3, 2)
    for _ in range(2):
        res["dma_h2d_ms"] = t(lambda: din.copy_(hin, non_blocking=True))
        res["dma_d2h_ms"] = t(lambda: hout.copy_(dout, non_blocking=True))

        def both():
            with torch.cuda.stream(s1):
                din.copy_(hin, non_blocking=True)
            with torch.cuda.stream(s2):
                hout.copy_(dout, non_blocking=True)
        res["dma_both_ms"] = t(both)
print(json.dumps(res))
