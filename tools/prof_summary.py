"""Summarise tools/gpu_profile.sh output (gpurun_out/prof) into profiles/.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim),
profiles/<tag>_k_decode.json (k_decode durations, HBM bytes, SQ counters)
and profiles/pmc_latest.json (read by bench.py for roofline.traffic).
HBM bytes per decode = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE counts half the bytes of a coalesced read (MI355X_MICROARCH.md, HBM).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")
KERNEL = "k_decode"


def find(sub, pat):
    hits = glob.glob(os.path.join(PROF, sub, "**", pat), recursive=True)
    if not hits:
        raise SystemExit(f"no {pat} under {sub}")
    return hits[0]


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def big(vals):
    """The bench-sized dispatches: the run also decodes the small kjv.txt
    source once (synth.load_source), which is not the measured workload."""
    m = max(vals)
    return [v for v in vals if v > 0.5 * m]


def counters(sub):
    """{counter: [value per bench-sized k_decode dispatch]} (summed over the
    per-dimension rows rocprofv3 writes for one dispatch)"""
    per = {}
    for r in rows(find(sub, "*counter_collection.csv")):
        if KERNEL not in r.get("Kernel_Name", ""):
            continue
        key = (r["Counter_Name"], r.get("Dispatch_Id", ""))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (name, _), v in per.items():
        out.setdefault(name, []).append(v)
    sizes = out.get("SQ_WAVE_CYCLES") or out.get("FETCH_SIZE") or out.get("WRITE_SIZE")
    if sizes:
        keep = [i for i, v in enumerate(sizes) if v > 0.5 * max(sizes)]
        out = {k: [v[i] for i in keep] for k, v in out.items()}
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    workload = sys.argv[2] if len(sys.argv) > 2 else "synthetic 1024 MiB/GPU kjv-tiled .huff"
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = find("kt", "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    kt = [r for r in rows(find("kt", "*kernel_trace.csv")) if KERNEL in r["Kernel_Name"]]
    dur = big([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in kt])
    fetch = counters("fetch").get("FETCH_SIZE", [])
    write = counters("write").get("WRITE_SIZE", [])
    sq = {k: statistics.mean(v) for k, v in counters("sq").items()}
    res = {"workload": workload, "kernel": KERNEL, "dispatches": len(dur),
           "ms_mean": statistics.mean(dur), "ms_min": min(dur), "ms_max": max(dur)}
    if fetch and write:
        fb = statistics.mean(fetch) * 1024 * 2
        wb = statistics.mean(write) * 1024
        res.update({"fetch_bytes_corrected": fb, "write_bytes": wb,
                    "hbm_bytes_per_decode": fb + wb,
                    "fetch_size_kib_raw": statistics.mean(fetch),
                    "write_size_kib_raw": statistics.mean(write)})
    res["sq"] = sq
    with open(os.path.join(ROOT, "profiles", f"{tag}_k_decode.json"), "w") as f:
        json.dump(res, f, indent=1)
    if "hbm_bytes_per_decode" in res:
        with open(os.path.join(ROOT, "profiles", "pmc_latest.json"), "w") as f:
            json.dump({"workload": workload, "hbm_bytes_per_decode": res["hbm_bytes_per_decode"],
                       "source": f"profiles/{tag}_k_decode.json"}, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
