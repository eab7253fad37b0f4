"""Summarise tools/profile.sh output (gpurun_out/prof/<tag>) into profiles/.

    python tools/prof_summary.py <tag> [workload]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<tag>_kernels.json: per kernel of the decode pipeline (k_front,
k_scan1, k_scan2, k_emit) the mean dispatch duration, HBM bytes per dispatch
and the SQ counters, over the bench-sized dispatches (those at least half as
long as the longest of that kernel).  HBM bytes per dispatch = 2 x FETCH_SIZE
+ WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE counts half the bytes of a
coalesced read (MI355X_MICROARCH.md, HBM).  Also writes
profiles/pmc_latest.json (read by bench.py for roofline.traffic: the whole
pipeline's bytes per decode).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_front", "k_walk", "k_table", "k_scan1", "k_scan2", "k_emitx", "k_emit", "k_cntm", "k_cnt", "k_fscan1", "k_fscan2", "k_emf")   # (k_emitx before k_emit: names match by substring)


def kname(s):
    for k in KERNELS:
        if k in s:
            return k
    return None


def csvs(prof, sub, pat):
    return glob.glob(os.path.join(prof, sub, "**", pat), recursive=True)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    workload = sys.argv[2] if len(sys.argv) > 2 else "synthetic 1024 MiB/GPU kjv-tiled .huff"
    prof = os.path.join(ROOT, "gpurun_out", "prof", tag)
    out_dir = os.path.join(ROOT, "profiles")
    stats = csvs(prof, "kt", "*kernel_stats.csv")
    if stats:
        shutil.copy(stats[0], os.path.join(out_dir, f"{tag}_kernel_stats.csv"))
    # durations per dispatch
    dur = {}
    for path in csvs(prof, "kt", "*kernel_trace.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = kname(r["Kernel_Name"])
                if k:
                    dur.setdefault(k, []).append(
                        (int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
    res = {"tag": tag, "workload": workload, "kernels": {}}
    for k, v in dur.items():
        big = max(d for _, d in v)
        keep = [d for _, d in v if d >= 0.5 * big]
        res["kernels"][k] = {"dispatches": len(keep), "ms_mean": round(statistics.mean(keep), 4),
                             "ms_min": round(min(keep), 4), "ms_max": round(max(keep), 4)}
    # counters: per kernel, the values of the bench-sized dispatches
    for sub in ("fetch", "write", "sq1", "sq2"):
        per = {}
        for path in csvs(prof, sub, "*counter_collection.csv"):
            with open(path) as f:
                for r in csv.DictReader(f):
                    k = kname(r.get("Kernel_Name", ""))
                    if not k:
                        continue
                    key = (k, r["Counter_Name"], path, r.get("Dispatch_Id", ""))
                    per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        by = {}
        for (k, name, _, _), v in per.items():
            by.setdefault((k, name), []).append(v)
        for (k, name), vs in by.items():
            top = max(vs)
            keep = [x for x in vs if x >= 0.5 * top] or vs
            res["kernels"].setdefault(k, {})[name] = statistics.mean(keep)
    tot_bytes = 0.0
    for k, d in res["kernels"].items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes"] = 1024.0 * (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"])
            tot_bytes += d["hbm_bytes"]
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            d["wait_frac"] = round(d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"], 3)
            d["active_frac"] = round(d.get("SQ_ACTIVE_INST_ANY", 0) / d["SQ_WAVE_CYCLES"], 3)
    res["hbm_bytes_per_decode"] = tot_bytes or None
    # FETCH_SIZE calibration on known byte counts (build/ub_fetch: 1 GiB read
    # with 16-B per-lane loads and with 4-B per-lane loads): bytes per KiB
    # counted, for each load shape; the decoder's kernels read the payload
    # with 16-B loads and their records with 4-B loads
    cal = {}
    for path in csvs(prof, "cal", "*counter_collection.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                n = r.get("Kernel_Name", "")
                key = "read16" if "k_read16" in n else "read4" if "k_read4" in n else None
                if key and r["Counter_Name"] == "FETCH_SIZE":
                    cal[key] = cal.get(key, 0.0) + float(r["Counter_Value"])
    if cal:
        res["fetch_calibration"] = {k: {"fetch_kib": v, "bytes_read": 1 << 30,
                                        "bytes_per_fetch_kib": round((1 << 30) / (v * 1024.0), 3)}
                                    for k, v in cal.items()}
    with open(os.path.join(out_dir, f"{tag}_kernels.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    if tot_bytes and len(sys.argv) <= 2:     # (the headline workload only: bench.py reads it)
        with open(os.path.join(out_dir, "pmc_latest.json"), "w") as f:
            json.dump({"workload": workload, "tag": tag, "hbm_bytes_per_decode": tot_bytes,
                       "per_kernel": {k: d.get("hbm_bytes") for k, d in res["kernels"].items()},
                       "fetch_calibration": res.get("fetch_calibration")},
                      f, indent=1)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
