# 64 MiB: count-kernel duration by regions per lane (kernel trace, no phase events)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
export HH_NO_PHASES=1
for m in 1 2 4; do
  for mib in 64 1024; do
    HH_CNT_M=$m timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/ktm_${m}_$mib -o run -- python3 tools/time_lib.py $mib 10 > $O/ktm.log 2>&1 || { tail -5 $O/ktm.log; exit 1; }
    echo "M=$m $mib MiB $(python3 tools/kt_sum.py $O/ktm_${m}_$mib | tr -d '\n ' | sed 's/.*"ms_span"/"ms_span"/')"
  done
done
