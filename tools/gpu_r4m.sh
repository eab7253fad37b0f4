# dynamic count-tile schedule: GPU tests, A/B at 64 MiB and 1 GiB against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -3 $O/t.log
export HH_NO_PHASES=1
MIB=64 ROUNDS=3 timeout -k 10 300 bash tools/gpu_ab.sh prev - > $O/ab64.log 2>&1; cat $O/ab64.log
ROUNDS=2 timeout -k 10 300 bash tools/gpu_ab.sh prev - > $O/ab.log 2>&1; cat $O/ab.log
SRC=bytes ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh prev - > $O/abb.log 2>&1; cat $O/abb.log
