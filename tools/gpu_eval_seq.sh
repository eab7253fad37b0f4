cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/eval
timeout -k 10 300 python3 tools/time_eval_seq.py > gpurun_out/eval/seq.json 2> gpurun_out/eval/seq.err; rc=$?; cat gpurun_out/eval/seq.json; exit $rc
