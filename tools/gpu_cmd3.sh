cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 150 python3 tools/diag_fsm.py paper1 > gpurun_out/d1.log 2>&1; echo "diag rc=$?"; tail -3 gpurun_out/d1.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "fixture or tiled or random or fixed or synthetic" > gpurun_out/t3.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t3.log
[ $rc -ge 124 ] && exit 1
bash tools/gpu_ab.sh "c1" "-" "- HH_EMF_NCH=1" "- HH_FSM_K=6" "- HH_FSM_K=6 HH_EMF_NCH=1" "c1w6" "c1w8" > gpurun_out/ab3.txt 2>&1; cat gpurun_out/ab3.txt
