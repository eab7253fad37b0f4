# LDS / VALU counters of the decode's kernels (1 GiB kjv-tiled, tools/time_lib.py)
# and of the LDS-chain microbenchmark at saturation (calibration of
# SQ_LDS_IDX_ACTIVE).  Passes of <= 8 SQ counters each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05}
R=gpurun_out/pmc/$TAG
rm -rf $R; mkdir -p $R
P1="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
run() { local n=$1; local what=$2; shift 2; echo "[$(date +%T)] $n"
  timeout -k 10 240 rocprofv3 $what --output-format csv -d $R/$n -o run -- "$@" > $R/$n.log 2>&1 || { tail -20 $R/$n.log; exit 1; }; }
run dec1 "--pmc $P1" python3 tools/time_lib.py 1024 3 kjv.txt
run dec2 "--pmc $P2" python3 tools/time_lib.py 1024 3 kjv.txt
run ub16 "--pmc $P1" build/ub_lds 1000 16 2
run ub16b "--pmc $P1" build/ub_lds 1000 16 8
run ub8 "--pmc $P1" build/ub_lds 1000 8 2
run kt "--kernel-trace --stats" python3 tools/time_lib.py 1024 5 kjv.txt
echo "[$(date +%T)] done main"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt64 -o run -- python3 tools/time_lib.py 64 5 kjv.txt > $R/kt64.log 2>&1 || { tail -20 $R/kt64.log; exit 1; }
echo "[$(date +%T)] done64"
