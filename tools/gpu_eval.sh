# evaluate() scope on the 1 GiB stream: host buffers first touched on the
# GPU's NUMA node, on the other node, and wherever the process runs
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/eval
for a in local remote none; do
  if [ $a = none ]; then unset HH_EVAL_AFFINITY; else export HH_EVAL_AFFINITY=$a; fi
  HH_EVAL_FLAGS=32 timeout -k 10 200 python3 tools/time_eval.py 1024 6 > gpurun_out/eval/$a.json 2>&1 && cat gpurun_out/eval/$a.json || exit 1
done
cat /proc/self/status | grep -i "cpus_allowed_list\|mems_allowed_list"
numactl -H 2>/dev/null | head -5 || true
