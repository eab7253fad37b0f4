# GPU-active cycles beside each dispatch's duration in ONE run (--pmc with
# --kernel-trace): the effective clock of each decode kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=gpurun_out/pmc/${1:-clk}
rm -rf $R; mkdir -p $R
timeout -k 10 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $R/a -o run -- python3 tools/time_lib.py 1024 3 kjv.txt > $R/a.log 2>&1 || { tail -20 $R/a.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $R/u -o run -- build/ub_lds 1000 16 2 > $R/u.log 2>&1 || { tail -20 $R/u.log; exit 1; }
echo done
