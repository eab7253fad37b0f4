cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 150 python3 tools/diag_fsm.py kjv.txt > gpurun_out/d19.log 2>&1; echo "diag rc=$?"; grep "gpu n" gpurun_out/d19.log
ROUNDS=2 bash tools/gpu_ab.sh "-" "head" "w8cw16" "w7cw14" > gpurun_out/ab19.txt 2>&1; cat gpurun_out/ab19.txt
