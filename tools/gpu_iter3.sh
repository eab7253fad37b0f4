# parity of the first build/ab library (HIPHUFF_LIB), then A/B timing of build/ab/*.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L0=$GRAFT_REPO_ROOT/$(ls build/ab/*.so | head -1)
HIPHUFF_LIB=$L0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in build/ab/*.so; do
    HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/time_lib.py 1024 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
