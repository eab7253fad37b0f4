# rocprofv3 evidence for the bench workload: kernel trace + stats, then HBM
# counters in their own passes (FETCH_SIZE and WRITE_SIZE cannot share one),
# then SQ stall counters.  Summaries land in gpurun_out/prof; copy with
# tools/prof_summary.py into profiles/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/prof
rm -rf $R; mkdir -p $R
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
echo "[$(date +%T)] kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o run -- $B > $R/kt.log 2>&1 || { tail -20 $R/kt.log; exit 1; }
tail -1 $R/kt.log
echo "[$(date +%T)] FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/fetch.log 2>&1 || { tail -20 $R/fetch.log; exit 1; }
echo "[$(date +%T)] WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/write.log 2>&1 || { tail -20 $R/write.log; exit 1; }
echo "[$(date +%T)] SQ counters"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $R/sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/sq.log 2>&1 || { tail -20 $R/sq.log; exit 1; }
echo "[$(date +%T)] done"
find $R -name "*.csv" | head -20
