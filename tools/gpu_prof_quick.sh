# Per-kernel device time of the decode pipeline (rocprofv3 kernel trace) on
# the 1 GiB kjv-tiled stream, plus the diagnostic build's phase fractions
# (build it first: make variant V=diag HIPEXTRA=-DHH_DIAG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SRC=${SRC:-kjv.txt}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq -o run -- python3 tools/time_lib.py ${MIB:-1024} 5 $SRC > gpurun_out/pq.log 2>&1 || { tail -20 gpurun_out/pq.log; exit 1; }
tail -1 gpurun_out/pq.log
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/pq/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-40s calls %4s avg %8.1f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
HH_DIAG=1 HIPHUFF_LIB=build/libhiphuff_diag.so timeout -k 10 180 python3 tools/time_lib.py ${MIB:-1024} 3 $SRC || exit 1
