# payload loads: plain vs nt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
export HH_NO_PHASES=1
ROUNDS=3 timeout -k 10 400 bash tools/gpu_ab.sh "-" "ldnt" > $O/ab.log 2>&1; cat $O/ab.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fixed" --timeout 120 --timeout-method thread > $O/t.log 2>&1; tail -1 $O/t.log
