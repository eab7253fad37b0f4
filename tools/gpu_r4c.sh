# GPU tests, then same-box A/B of the previous commit (build/var/prev.so)
# against the working tree on the kjv and E.coli (state machine) streams.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -3 $O/t.log
ROUNDS=2 timeout -k 10 300 bash tools/gpu_ab.sh prev - "- HH_EMF_SCO=0" > $O/ab.log 2>&1; cat $O/ab.log
SRC=E.coli ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh "prev HH_FLAGS=4" "- HH_FLAGS=4" > $O/ab_ecoli.log 2>&1; cat $O/ab_ecoli.log
