"""A/B timing (tools/gpu_ab.sh): the decode pipeline on the synthetic stream with
the library named by HIPHUFF_LIB (default: the in-tree build); prints one
JSON line with the median device time of each kernel phase over N runs and
whether the output matched the tiled text.

    python tools/time_lib.py [MiB] [runs] [source]   (source: kjv.txt | E.coli | bytes | iid)
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

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
src = sys.argv[3] if len(sys.argv) > 3 else "kjv.txt"
# the source text comes from the in-tree library (the A/B scripts cache it), so
# that an experiment variant under test never decodes its own reference
cache = os.environ.get("HH_TEXT_CACHE")
if src == "bytes":
    # bench's byte-alphabet workload: generated and encoded on the GPU,
    # checked against its symbols (no text to cache)
    hf = text = None
elif src == "iid":
    # bench's i.i.d. kjv-unigram workload (symbols checked against the generator)
    hf0, text0 = synth.load_source(os.path.join(ROOT, "files"), "kjv.txt")
    hf = text = None
elif cache and os.path.exists(cache):
    import numpy as np
    hf = H.HuffFile.load(os.path.join(ROOT, "files", src + ".huff"))
    text = np.load(cache)
else:
    hf, text = synth.load_source(os.path.join(ROOT, "files"), src)
    if cache:
        import numpy as np
        np.save(cache, text)
        sys.exit(0)
if src == "bytes":
    syn = synth.byte_stream(mib << 20)
elif src == "iid":
    syn = synth.iid_stream(hf0, text0, mib << 20)
else:
    syn = synth.tiled_stream(hf, text, mib << 20)


def verify(out, n):
    if hf is None:
        return n == syn.decoded_bytes and bool(torch.equal(out[:n], syn.syms))
    return n == syn.decoded_bytes and synth.verify_tiled(out, syn)
# (with the phase events between the kernels: the A/B tables report the split)
dec = H.Decoder(0, lane_bits=int(os.environ.get("HH_LANE_BITS", "0")),
                flags=int(os.environ.get("HH_FLAGS", "0")) | (0 if os.environ.get("HH_NO_PHASES") else H.FLAG_PHASE_TIMING))
dec.set_tree(syn.tree)
out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
ph = {"total": [], "sync": [], "scan": [], "emit": []}
wall = []
ok = True
for i in range(reps + 1):
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        n = dec.decode_device(syn.data, syn.bits, out)
    except H.HipHuffError:          # experiment variants (wrong counts by design)
        n = -1
    torch.cuda.synchronize()
    wall.append((time.perf_counter() - t0) * 1e3)
    if i == 0:
        ok = verify(out, n)
        continue
    st = dec.stats()
    for k in ph:
        ph[k].append(st["ms_" + k])
res = {"lib": os.path.basename(os.environ.get("HIPHUFF_LIB", H.LIB_PATH)), "mib": mib, "src": src,
       "ok": bool(ok), "fast": dec.stats()["exact_fallback"] == 0}
res.update({k: round(statistics.median(v), 4) for k, v in ph.items()})
res["wall_ms"] = round(statistics.median(wall[1:]), 3)
if os.environ.get("HH_DIAG"):              # a -DHH_DIAG build (round 2 pipeline): phase cycles and walk lengths
    import ctypes as C
    buf = (C.c_uint64 * 16)()
    H.lib().hh_debug_counters(dec._h, buf)
    cyc = [buf[i] for i in range(6)]
    tot = sum(cyc) or 1
    res["front_phase_frac"] = {n: round(cyc[i] / tot, 3) for n, i in
                               (("stage", 0), ("pass1", 1), ("merge_defer", 2), ("records", 3))}
    ecyc = [buf[i] for i in (6, 7, 12, 13, 14)]
    etot = sum(ecyc) or 1
    res["emit_phase_frac"] = {n: round(v / etot, 3) for n, v in
                              zip(("records_scan", "zero", "decode", "decode_wait", "copyout"), ecyc)}
    if buf[8]:
        res["walk"] = {"mean_steps": round(buf[9] / buf[8], 2), "mean_wave_max": round(buf[10] / (buf[8] / 64), 2),
                       "max": buf[11]}
print(json.dumps(res), flush=True)
