cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v -k "shard_job" --timeout 200 --timeout-method thread > gpurun_out/t23.log 2>&1; rc=$?; echo "rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/t23.log | head -20
