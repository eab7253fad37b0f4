# parity, short bench, then the stamps diagnostic; stops at the first failing step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity.log 2>&1
rc=$?; cat gpurun_out/smoke.log; tail -3 gpurun_out/parity.log; echo "parity rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/libhiphuff_stamps.so timeout -k 10 200 python tools/diag_stamps.py 1024 > gpurun_out/stamps.log 2>&1; rc=$?; cat gpurun_out/stamps.log; exit $rc
