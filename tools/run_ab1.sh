set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "segment or resynchronising" > gpurun_out/t_seg.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not eight_shards and not hufx" > gpurun_out/t.log 2>&1 || exit 1
