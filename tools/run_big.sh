set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/tests_full.log 2>&1 || exit 1
timeout -k 10 600 python3 -u tools/sweep.py gpurun_out/size_sweep.json > gpurun_out/sweep.log 2>&1 || exit 1
timeout -k 10 120 build/HuffFramework graph2 --files files > gpurun_out/graph2.txt 2> gpurun_out/graph2.err || exit 1
timeout -k 10 120 build/HuffFramework quickgraph2 --files files > gpurun_out/quickgraph2.txt 2>> gpurun_out/graph2.err || exit 1
