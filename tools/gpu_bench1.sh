set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
cat gpurun_out/bench1.json
tail -5 gpurun_out/bench1.err
