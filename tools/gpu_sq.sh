# SQ counters of the bench workload in two passes (<= 8 SQ counters each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/sq
rm -rf $R; mkdir -p $R
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
echo "[$(date +%T)] SQ pass A"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/a -o run -- python3 $B > $R/a.log 2>&1 || { tail -20 $R/a.log; exit 1; }
echo "[$(date +%T)] SQ pass B"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA --output-format csv -d $R/b -o run -- python3 $B > $R/b.log 2>&1 || { tail -20 $R/b.log; exit 1; }
echo "[$(date +%T)] done"
python3 tools/sq_summary.py $R
