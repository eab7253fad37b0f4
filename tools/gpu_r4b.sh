# Round-4 GPU experiments: k_cnt phase cycles (HH_DIAG build), region size
# and emission step, heads of 96 / 128 bits.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
HH_DIAG=fsm HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/var/diag.so timeout -k 10 120 python3 tools/time_lib.py 1024 3 > $O/diag.json 2>&1; cat $O/diag.json
ROUNDS=2 timeout -k 10 500 bash tools/gpu_ab.sh - "- HH_LANE_BITS=384 HH_FSM_K=7" "- HH_LANE_BITS=384" "- HH_FSM_HEAD=96" "- HH_LANE_BITS=320 HH_FSM_K=7" > $O/ab.log 2>&1; cat $O/ab.log
