# A/B timing (tools/gpu_ab.sh) plus a WRITE_SIZE and a FETCH_SIZE pass per library
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_ab.sh || exit 1
for L in build/ab/*.so; do
  n=$(basename $L .so)
  for C in WRITE_SIZE FETCH_SIZE; do
    HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/abpmc/$n/$C -o run -- python3 tools/time_lib.py 1024 2 > /dev/null 2>&1 || { echo "pmc $n $C failed"; exit 1; }
  done
  python3 - "$n" <<'PY'
import csv, glob, sys
n = sys.argv[1]
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    vals = {}
    for p in glob.glob(f"gpurun_out/abpmc/{n}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "k_decode" in r["Kernel_Name"]:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    v = sorted(vals.values())
    print(f"{n} {c}: max dispatch {v[-1] * 1024 / 1e9:.3f} GB (KiB x 1024)" if v else f"{n} {c}: none")
PY
done
