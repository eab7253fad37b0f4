# head length A/B with 2 regions per count lane
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
ROUNDS=2 timeout -k 10 400 bash tools/gpu_ab.sh "-" "- HH_FSM_HEAD=96" "- HH_FSM_HEAD=112" "- HH_FSM_HEAD=80" > $O/ab.log 2>&1; cat $O/ab.log
SRC=bytes ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh "-" "- HH_FSM_HEAD=98" "- HH_FSM_HEAD=112" > $O/abb.log 2>&1; cat $O/abb.log
