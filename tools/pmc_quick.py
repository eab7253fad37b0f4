"""Per-kernel means of one rocprofv3 --pmc run (counter_collection.csv under
DIR), over the dispatches at least half as large as the largest of that
kernel, with a few derived per-instruction figures.
    python3 tools/pmc_quick.py DIR"""
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("k_cntm", "k_cnt", "k_fscan1", "k_fscan2", "k_emf", "k_fixed", "k_one")
per = {}
for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r.get("Kernel_Name", "")
            k = next((x for x in KERNELS if x in n), None)
            if not k:
                continue
            key = (k, r["Counter_Name"], path, r.get("Dispatch_Id", ""))
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
by = {}
for (k, name, _, _), v in per.items():
    by.setdefault((k, name), []).append(v)
res = {}
for (k, name), vs in by.items():
    top = max(vs)
    keep = [x for x in vs if x >= 0.5 * top] or vs
    res.setdefault(k, {})[name] = statistics.mean(keep)
for k, d in res.items():
    n = d.get("SQ_INSTS_LDS")
    if n:
        if "SQ_LDS_BANK_CONFLICT" in d:
            d["conflict_per_lds_inst"] = round(d["SQ_LDS_BANK_CONFLICT"] / n, 2)
        if "SQ_LDS_IDX_ACTIVE" in d:
            d["lds_cycles_per_inst"] = round(d["SQ_LDS_IDX_ACTIVE"] / n, 2)
    if d.get("SQ_BUSY_CYCLES") and "SQ_LDS_IDX_ACTIVE" in d:
        d["lds_idx_active_per_busy"] = round(d["SQ_LDS_IDX_ACTIVE"] / d["SQ_BUSY_CYCLES"], 3)
    if d.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
            if c in d:
                d[c.lower() + "_frac"] = round(d[c] / d["SQ_WAVE_CYCLES"], 3)
print(json.dumps(res, indent=1, sort_keys=True))
