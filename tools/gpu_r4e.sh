set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -2 $O/t.log
SRC=E.coli ROUNDS=2 timeout -k 10 300 bash tools/gpu_ab.sh "- HH_FLAGS=4" "- HH_FLAGS=4 HH_EMF_SWZ=0" > $O/ab_ecoli.log 2>&1; cat $O/ab_ecoli.log
ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh - "- HH_EMF_SWZ=1" > $O/ab.log 2>&1; cat $O/ab.log
