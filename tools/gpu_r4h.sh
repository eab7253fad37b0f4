# Round-4: full GPU tests with the count pass at 2 regions per lane; M=1/2/4
# on kjv and the byte alphabet; the byte alphabet's emission step width.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -3 $O/t.log
ROUNDS=2 timeout -k 10 300 bash tools/gpu_ab.sh "- HH_CNT_M=1" "- HH_CNT_M=2" "- HH_CNT_M=4" > $O/ab.log 2>&1; cat $O/ab.log
SRC=bytes ROUNDS=1 timeout -k 10 400 bash tools/gpu_ab.sh "- HH_CNT_M=2" "- HH_CNT_M=4" "- HH_CNT_M=4 HH_FSM_K=5" "- HH_CNT_M=4 HH_FSM_K=4" > $O/abb.log 2>&1; cat $O/abb.log
SRC=E.coli ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh "- HH_FLAGS=4 HH_CNT_M=1" "- HH_FLAGS=4 HH_CNT_M=2" "- HH_FLAGS=4 HH_CNT_M=4" > $O/abe.log 2>&1; cat $O/abe.log
for mib in 64 1024; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$mib -o run -- python3 tools/time_lib.py $mib 20 > $O/kt_$mib.log 2>&1 || { tail -5 $O/kt_$mib.log; exit 1; }
  echo "== kernel trace $mib MiB"; python3 tools/kt_sum.py $O/kt_$mib
done
