# count-pass occupancy A/B (M=2 at 28 waves per CU vs 24)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
ROUNDS=2 timeout -k 10 300 bash tools/gpu_ab.sh "-" "v14" > $O/ab.log 2>&1; cat $O/ab.log
SRC=bytes ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh "-" "v14" > $O/abb.log 2>&1; cat $O/abb.log
