# Round-3 state-machine path: microbenchmark, 1 GiB kjv timing (new vs legacy),
# GPU parity suite.  Every GPU step under its own time limit, chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./build/ub_fsm > gpurun_out/ub_fsm.log 2>&1 && \
timeout -k 10 240 python3 tools/time_lib.py 1024 5 kjv.txt > gpurun_out/t_fsm.log 2>&1 && \
HH_FLAGS=8 timeout -k 10 240 python3 tools/time_lib.py 1024 5 kjv.txt > gpurun_out/t_legacy.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
cat gpurun_out/ub_fsm.log; tail -1 gpurun_out/t_fsm.log; tail -1 gpurun_out/t_legacy.log; tail -15 gpurun_out/gputests.log
exit $rc
