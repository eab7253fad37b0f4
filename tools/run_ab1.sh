set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not eight_shards and not hufx" > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2> gpurun_out/bench.err || exit 1
