cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t17.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t17.log
[ $rc -ge 124 ] && exit 1
MIB=64 ROUNDS=3 bash tools/gpu_ab.sh "-" "head" "- HH_EMF_NOSCO=1" > gpurun_out/ab17s.txt 2>&1; cat gpurun_out/ab17s.txt
ROUNDS=2 bash tools/gpu_ab.sh "-" "head" "- HH_EMF_NOSCO=1" > gpurun_out/ab17.txt 2>&1; cat gpurun_out/ab17.txt
