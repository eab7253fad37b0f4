# Round-3 state-machine path on one GPU: diagnostics against the emulator,
# 1 GiB kjv timing (new vs legacy pipeline), the GPU parity suite.  Every
# GPU step under its own time limit; a crash, abort or timeout (exit >= 124)
# ends the script, a wrong answer (exit 1) does not.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {   # name, limit, command...
    local name=$1 lim=$2; shift 2
    timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -${TAILN:-12} gpurun_out/$name.log
    if [ $rc -ge 124 ]; then exit $rc; fi
    return 0
}
for f in ${DIAG:-hello paper1 kjv.txt}; do step diag_$f 150 python3 tools/diag_fsm.py $f; done
[ -n "$NOTIME" ] || step t_fsm 240 python3 tools/time_lib.py 1024 5 kjv.txt
[ -n "$NOTIME" ] || HH_FLAGS=8 step t_legacy 240 python3 tools/time_lib.py 1024 5 kjv.txt
[ -n "$NOTIME" ] || step e_pipe 240 python3 tools/time_eval.py 1024 5
[ -n "$NOTIME" ] || HH_PIPE_CHUNK_KB=32768 step e_pipe32 240 python3 tools/time_eval.py 1024 5
[ -n "$NOTIME" ] || HH_HOST_SERIAL=1 step e_serial 240 python3 tools/time_eval.py 1024 3
[ -n "$NOTEST" ] || TAILN=25 step gputests 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
exit 0
