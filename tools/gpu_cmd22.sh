cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t22.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t22.log
[ $rc -ge 124 ] && exit 1
ROUNDS=2 bash tools/gpu_ab.sh "-" "head" > gpurun_out/ab22.txt 2>&1; cat gpurun_out/ab22.txt
export HH_FLAGS=4
SRC=E.coli ROUNDS=2 bash tools/gpu_ab.sh "-" "- HH_FSM_K=7" > gpurun_out/ab22e.txt 2>&1; cat gpurun_out/ab22e.txt
