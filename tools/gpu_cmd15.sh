cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for f in paper1 kjv.txt; do timeout -k 10 150 python3 tools/diag_fsm.py $f > gpurun_out/d15_$f.log 2>&1; echo "diag $f rc=$?"; grep -E "gpu n" gpurun_out/d15_$f.log; done
ROUNDS=2 bash tools/gpu_ab.sh "-" "pnx0" "diag HH_DIAG=fsm" > gpurun_out/ab15.txt 2>&1; cat gpurun_out/ab15.txt
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t15.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/t15.log
