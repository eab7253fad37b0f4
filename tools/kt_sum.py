"""Per-decode kernel time from a rocprofv3 --kernel-trace run (kernel_trace.csv
under DIR): the decodes are the groups of dispatches between consecutive
k_cnt main launches; reports the mean over the large decodes of the summed
kernel durations and of the first-start-to-last-end span (which includes
the gaps between the launches), beside the bench line's HIP-event
ms_kernel if a bench JSON is given.
    python3 tools/kt_sum.py DIR [bench.json]"""
import csv
import glob
import json
import os
import statistics
import sys

NAMES = ("k_cntm", "k_cnt", "k_fscan1", "k_fscan2", "k_emf", "k_fixed")
rows = []
for path in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            k = next((x for x in NAMES if x in n), None)
            if k:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, n))
rows.sort()
# a decode starts at each k_cnt whose predecessor was a k_emf (or the first)
decodes, cur = [], []
for r in rows:
    if r[2] in ("k_cnt", "k_cntm") and cur and cur[-1][2] == "k_emf":
        decodes.append(cur)
        cur = []
    cur.append(r)
if cur:
    decodes.append(cur)
sums = [sum(e - s for s, e, _, _ in d) * 1e-6 for d in decodes]
spans = [(d[-1][1] - d[0][0]) * 1e-6 for d in decodes]
big = max(sums) if sums else 0
keep = [i for i, v in enumerate(sums) if v >= 0.5 * big]
per_kernel = {}
for i in keep:
    for s, e, k, _ in decodes[i]:
        per_kernel.setdefault(k, []).append((e - s) * 1e-6)
# the idle time inside a decode: each gap between one kernel's end and the
# next one's start (launch order), and the gap before the next decode
gaps = {}
for i in keep:
    d = decodes[i]
    for a in range(1, len(d)):
        gaps.setdefault(a, []).append((d[a][0] - d[a - 1][1]) * 1e-3)
between = [(decodes[i + 1][0][0] - decodes[i][-1][1]) * 1e-3 for i in keep if i + 1 < len(decodes)]
res = {"decodes": len(keep),
       "launches_per_decode": round(statistics.mean(len(decodes[i]) for i in keep), 2),
       "gap_us_after_launch": {a: round(statistics.mean(v), 2) for a, v in gaps.items()},
       "gap_us_between_decodes": round(statistics.mean(between), 2) if between else None,
       "ms_kernel_sum": round(statistics.mean(sums[i] for i in keep), 4),
       "ms_span": round(statistics.mean(spans[i] for i in keep), 4),
       "per_decode_ms": {k: round(sum(v) / len(keep), 4) for k, v in per_kernel.items()}}
if len(sys.argv) > 2:
    with open(sys.argv[2]) as f:
        b = json.loads(f.read().strip().splitlines()[-1])
    r = b["roofline"]
    res["bench_ms_kernel"] = r["ms_kernel"]
    res["bench_frac"] = r["frac"]
    res["frac_from_trace_sum"] = round(r["bytes_alg"] / (res["ms_kernel_sum"] * 1e-3) / 1e9 / r["peak"], 4)
    res["frac_from_trace_span"] = round(r["bytes_alg"] / (res["ms_span"] * 1e-3) / 1e9 / r["peak"], 4)
print(json.dumps(res, indent=1))
