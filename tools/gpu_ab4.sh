# parity (full GPU parity file) of every build/ab/*.so, then 2 rounds of A/B timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in build/ab/*.so; do
  HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_$(basename $L).log 2>&1
  rc=$?; echo "$L parity: $(tail -1 gpurun_out/ab_$(basename $L).log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for L in build/ab/*.so; do
    HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/time_lib.py 1024 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
