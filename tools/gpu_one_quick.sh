# Single-pass quick check on the GPU box: correctness + timing (one_check.py)
# and the diagnostic counters (one_diag.py, the odbg variant build).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HH_ONE=1
timeout -k 10 240 python3 -u tools/one_check.py ${SIZES:-64 1024} > gpurun_out/oneq.log 2>&1 || { echo check failed; tail -5 gpurun_out/oneq.log; exit 1; }
cat gpurun_out/oneq.log | grep -v amdgpu.ids
if [ -f build/libhiphuff_odbg.so ]; then
  HIPHUFF_LIB=$PWD/build/libhiphuff_odbg.so HH_ONE_DBG=1 timeout -k 10 120 python3 -u tools/one_diag.py ${DMIB:-1024} 2>&1 | grep -v amdgpu.ids
fi
if [ -n "$LB2" ]; then
  HH_LANE_BITS=$LB2 ONE_FIXTURES=0 timeout -k 10 200 python3 -u tools/one_check.py 1024 2>&1 | grep -v amdgpu.ids
  HIPHUFF_LIB=$PWD/build/libhiphuff_odbg.so HH_ONE_DBG=1 HH_LANE_BITS=$LB2 timeout -k 10 120 python3 -u tools/one_diag.py 1024 2>&1 | grep -v amdgpu.ids
fi
