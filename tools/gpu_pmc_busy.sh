# Clock and SE-busy fractions of the decode's kernels: GRBM_GUI_ACTIVE (GPU
# busy cycles) and SQ_BUSY_CYCLES per dispatch, beside a kernel trace of the
# same program (durations).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05}
R=gpurun_out/pmc/$TAG
rm -rf $R; mkdir -p $R
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d $R/busy -o run -- python3 tools/time_lib.py 1024 3 kjv.txt > $R/busy.log 2>&1 || { tail -20 $R/busy.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/kt -o run -- python3 tools/time_lib.py 1024 3 kjv.txt > $R/kt.log 2>&1 || { tail -20 $R/kt.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d $R/ub -o run -- build/ub_lds 1000 16 2 > $R/ub.log 2>&1 || { tail -20 $R/ub.log; exit 1; }
echo done
