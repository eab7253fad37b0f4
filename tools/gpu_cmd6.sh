cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
HH_FSM_HEAD=128 timeout -k 10 150 python3 tools/diag_fsm.py kjv.txt > gpurun_out/d6.log 2>&1; echo "diag rc=$?"; tail -2 gpurun_out/d6.log
ROUNDS=2 bash tools/gpu_ab.sh "-" "- HH_FSM_HEAD=96" "- HH_FSM_HEAD=128" "- HH_FSM_HEAD=80" > gpurun_out/ab6.txt 2>&1; cat gpurun_out/ab6.txt
