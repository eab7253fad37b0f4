"""Print the mean of each SQ counter over the bench-sized k_decode dispatches
found under a directory of rocprofv3 --pmc outputs (tools/gpu_sq.sh)."""
import csv
import glob
import sys

root = sys.argv[1]
per = {}
for path in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            if "k_decode" not in r.get("Kernel_Name", ""):
                continue
            k = (r["Counter_Name"], path, r.get("Dispatch_Id", ""))
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
by = {}
for (name, _, _), v in per.items():
    by.setdefault(name, []).append(v)
for name, vs in sorted(by.items()):
    m = max(vs)
    big = [v for v in vs if v > 0.5 * m]
    print(f"{name:24s} {sum(big) / len(big):.4e}  (n={len(big)})")
