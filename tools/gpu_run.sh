# One GPU session: build check, the -m gpu suite, then a bench line.
#   bash tools/gpu_run.sh TAG [tests|bench|all]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05}
WHAT=${2:-all}
E=gpurun_out/$TAG
mkdir -p $E
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  echo "[$(date +%T)] tests"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $E/gpu_tests.log 2>&1 || { tail -30 $E/gpu_tests.log; exit 1; }
  tail -1 $E/gpu_tests.log
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  echo "[$(date +%T)] bench"
  timeout -k 10 600 python3 bench.py > $E/bench.json 2> $E/bench.err || { tail -20 $E/bench.err; exit 1; }
  cat $E/bench.json
fi
echo "[$(date +%T)] done"
