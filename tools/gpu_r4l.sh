# byte alphabet: count-pass workgroup width for 7-bit count steps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
SRC=bytes ROUNDS=2 timeout -k 10 400 bash tools/gpu_ab.sh "-" "c7w12" "- HH_CNT_M=4" > $O/abb.log 2>&1; cat $O/abb.log
