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
if os.environ.get("HH_WSPAN"):             # a -DHH_WSPAN build: per-wave start / fill / end (100 MHz clock)
    import ctypes as C
    import numpy as np
    N = 8192
    buf = (C.c_uint64 * (16 + 10 * N))()
    H.lib().hh_debug_counters(dec._h, buf)
    a = np.ctypeslib.as_array(buf)[16:].astype(np.int64)
    if os.environ.get("HH_WSPAN_DUMP"):
        np.save(os.environ["HH_WSPAN_DUMP"] + f"_{mib}.npy", a)
    for name, o in (("cnt", 0), ("emf", 3 * N)):
        st = a[o:o + 3 * N].reshape(N, 3).copy()
        st = st[st[:, 2] > 0]
        if not len(st):
            continue
        ev = st[:, 1] >> 48                    # (events in the fill stamp's top bits: walk rounds, fixes << 10)
        st[:, 1] &= (1 << 48) - 1
        t0 = st[:, 0].min()
        us = lambda x: np.round(np.asarray(x) / 100.0, 2).tolist()   # noqa: E731  (100 MHz ticks -> us)
        dur = st[:, 2] - st[:, 0]
        ends = np.sort(st[:, 2] - t0)
        res[name + "_span"] = {"waves": int(len(st)), "kernel_us": us(ends[-1]),
                               "start_spread_us": us(st[:, 0].max() - t0),
                               "fill_us_mean": us((st[:, 1] - st[:, 0]).mean()),
                               "wave_us_p0_p50_p90_p99_max": us(np.percentile(dur, [0, 50, 90, 99, 100])),
                               "end_us_p1_p10_p50_p90_max": us(np.percentile(ends, [1, 10, 50, 90, 100]))}
        if name == "cnt":                      # (k_cntm's per-wave phase ticks: heads, counts, walks, the rest)
            ph = a[6 * N:10 * N].reshape(N, 4)[np.nonzero(a[2:3 * N:3] > 0)[0]]
            tot = ph.sum(axis=1).clip(min=1)
            res[name + "_span"]["phase_frac_heads_counts_walks_rest"] = np.round(ph.sum(axis=0) / tot.sum(), 4).tolist()
        if ev.any():
            rounds, fixes = ev & 1023, ev >> 10
            slow = np.argsort(st[:, 2] - st[:, 0])[-20:]
            res[name + "_span"].update({"walk_rounds_total": int(rounds.sum()), "walk_rounds_p50_p99_max":
                                        np.percentile(rounds, [50, 99, 100]).tolist(), "fixes_total": int(fixes.sum()),
                                        "slowest20_rounds": rounds[slow].tolist(), "slowest20_fixes": fixes[slow].tolist()})
elif os.environ.get("HH_DIAG") == "fsm":     # a -DHH_DIAG build: k_cnt phase cycles and walks
    import ctypes as C
    buf = (C.c_uint64 * 16)()
    H.lib().hh_debug_counters(dec._h, buf)
    cyc = [buf[i] for i in range(4)]
    tot = sum(cyc) or 1
    res["cnt_phase_frac"] = {n: round(cyc[i] / tot, 3) for n, i in
                             (("head", 0), ("count", 1), ("walks", 2), ("records", 3))}
    res["cnt_tiles"] = buf[8]
    res["cnt_walk_tiles"] = buf[9]
    res["cnt_walk_rounds"] = buf[10]
    res["cnt_cycles_per_tile"] = round(tot / max(buf[8], 1), 1)
    ecyc = [buf[i] for i in range(4, 8)]
    etot = sum(ecyc) or 1
    res["emf_phase_frac"] = {n: round(ecyc[i] / etot, 3) for n, i in
                             (("prologue", 0), ("region", 1), ("edges", 2), ("copyout", 3))}
    res["emf_cycles_per_tile"] = round(etot / max(buf[8], 1), 1)
elif os.environ.get("HH_DIAG"):            # a -DHH_DIAG build: phase cycles and walk lengths
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
