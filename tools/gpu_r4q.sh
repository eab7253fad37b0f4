# k_emf copy-out stores: plain vs nt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
export HH_NO_PHASES=1
ROUNDS=3 timeout -k 10 400 bash tools/gpu_ab.sh "-" "nt" > $O/ab.log 2>&1; cat $O/ab.log
SRC=E.coli ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh "- HH_FLAGS=4" "nt HH_FLAGS=4" > $O/abe.log 2>&1; cat $O/abe.log
