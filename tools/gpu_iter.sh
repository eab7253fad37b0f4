# parity tests, the synthetic diagnostic and the phase stamps; stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/parity.log 2>&1
rc=$?; tail -4 gpurun_out/parity.log; echo "parity rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag_synth.py ${SIZES:-256 1024} > gpurun_out/diag_synth.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/diag_synth.txt | head -30; echo "synth rc=$rc"
[ $rc -eq 0 ] || exit $rc
HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/libhiphuff_stamps.so timeout -k 10 200 python tools/diag_stamps.py 1024 > gpurun_out/stamps.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/stamps.log; exit $rc
