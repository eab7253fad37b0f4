cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/eval
timeout -k 10 200 python3 tools/time_eval.py 1024 6 > gpurun_out/eval/a.json 2>&1 && cat gpurun_out/eval/a.json &&
HH_EVAL_FLAGS=32 HH_EVAL_DMA=1 timeout -k 10 200 python3 tools/time_eval.py 1024 6 > gpurun_out/eval/b.json 2>&1 && cat gpurun_out/eval/b.json &&
HH_HOST_SERIAL=1 timeout -k 10 200 python3 tools/time_eval.py 1024 4 > gpurun_out/eval/c.json 2>&1 && cat gpurun_out/eval/c.json
