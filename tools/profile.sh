# rocprofv3 evidence for the decode pipeline on the bench workload
# (tools/time_lib.py: the 1 GiB kjv-tiled stream, decoded RUNS+1 times):
# kernel trace + stats, then counters in passes of their own (FETCH_SIZE and
# WRITE_SIZE cannot share one; SQ counters in two passes of <= 8).  Outputs
# in gpurun_out/prof/<tag>; tools/prof_summary.py <tag> writes profiles/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
MIB=${MIB:-1024}
SRC=${SRC:-kjv.txt}
R=$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG
rm -rf $R; mkdir -p $R
P="python3 tools/time_lib.py $MIB 5 $SRC"
run() {   # name, rocprofv3 args...
  local n=$1; shift
  echo "[$(date +%T)] $n"
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $R/$n -o run -- $P > $R/$n.log 2>&1 || { tail -20 $R/$n.log; exit 1; }
  tail -1 $R/$n.log
}
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU
run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SMEM
# FETCH_SIZE calibration: 1 GiB read with 16-B and with 4-B per-lane loads
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/cal -o run -- build/ub_fetch > $R/cal.log 2>&1 || { tail -20 $R/cal.log; exit 1; }
echo "[$(date +%T)] done"
