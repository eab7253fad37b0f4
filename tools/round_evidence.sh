# Round-end evidence on one MI355X, everything under gpurun_out/evidence:
# the GPU test log, rocprofv3 kernel stats and counters (tools/profile.sh),
# the bench line (reading the fresh counters), a kernel trace of the bench
# itself (no counters: its per-decode kernel sum beside the bench's HIP-event
# time, tools/kt_sum.py), the 64 MiB .. 8 GiB size sweep and the reference's
# graph2/quickgraph2 curves.  Copy to profiles/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04}
E=gpurun_out/evidence
mkdir -p $E
echo "[$(date +%T)] tests"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $E/${TAG}_gpu_tests.log 2>&1 || { tail -20 $E/${TAG}_gpu_tests.log; exit 1; }
tail -1 $E/${TAG}_gpu_tests.log
echo "[$(date +%T)] profile"
bash tools/profile.sh $TAG > $E/profile.log 2>&1 || { tail -20 $E/profile.log; exit 1; }
python3 tools/prof_summary.py $TAG > $E/prof_summary.log 2>&1 || exit 1
cp profiles/${TAG}_kernels.json profiles/${TAG}_kernel_stats.csv profiles/pmc_latest.json $E/
echo "[$(date +%T)] bench"
timeout -k 10 600 python3 bench.py > $E/${TAG}_bench_latest.json 2> $E/bench.err || { tail -20 $E/bench.err; exit 1; }
cat $E/${TAG}_bench_latest.json
echo "[$(date +%T)] bench under a kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $E/kt_bench -o run -- python3 bench.py --no-extra --no-cpu-baseline > $E/${TAG}_bench_traced.json 2> $E/kt_bench.err || { tail -20 $E/kt_bench.err; exit 1; }
python3 tools/kt_sum.py $E/kt_bench $E/${TAG}_bench_latest.json > $E/${TAG}_bench_trace_sum.json && cat $E/${TAG}_bench_trace_sum.json
cp $(find $E/kt_bench -name "*kernel_stats.csv" | head -1) $E/${TAG}_bench_kernel_stats.csv
echo "[$(date +%T)] sweep"
timeout -k 10 600 python3 -u tools/sweep.py $E/${TAG}_size_sweep.json > $E/sweep.log 2>&1 || { tail -20 $E/sweep.log; exit 1; }
timeout -k 10 120 build/HuffFramework graph2 --files $(python3 tools/regen_files.py gpurun_out/files_full) > $E/${TAG}_graph2_hip.txt 2> $E/graph2.err || exit 1
timeout -k 10 120 build/HuffFramework quickgraph2 --files files > $E/${TAG}_quickgraph2_hip.txt 2>> $E/graph2.err || exit 1
echo "[$(date +%T)] done"
