cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/t16.log
[ $rc -ge 124 ] && exit 1
ROUNDS=2 bash tools/gpu_ab.sh "-" "- HH_EMF_NOSCO=1" > gpurun_out/ab16.txt 2>&1; cat gpurun_out/ab16.txt
MIB=64 ROUNDS=1 bash tools/gpu_ab.sh "-" > gpurun_out/ab16s.txt 2>&1; cat gpurun_out/ab16s.txt
