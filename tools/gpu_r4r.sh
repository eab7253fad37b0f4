# k_fixed output stores: plain vs nt (E.coli-tiled, k_fixed path); GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
export HH_NO_PHASES=1
SRC=E.coli ROUNDS=3 timeout -k 10 400 bash tools/gpu_ab.sh "-" "fnt" > $O/abe.log 2>&1; cat $O/abe.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -1 $O/t.log
