set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/profile.sh r02 > gpurun_out/profile.log 2>&1 || { tail -20 gpurun_out/profile.log; exit 1; }
python3 tools/prof_summary.py r02 "synthetic 1024 MiB/GPU kjv-tiled .huff" > gpurun_out/prof_summary.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || exit 1
