cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 150 python3 tools/diag_fsm.py kjv.txt > gpurun_out/d18.log 2>&1; echo "diag rc=$?"; grep "gpu n" gpurun_out/d18.log
ROUNDS=3 bash tools/gpu_ab.sh "-" "head" > gpurun_out/ab18.txt 2>&1; cat gpurun_out/ab18.txt
