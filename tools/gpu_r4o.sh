# count/emission kernel time against stream size (kernel trace, no phase events)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
export HH_NO_PHASES=1
for mib in 4 16 32 64 128; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/kts_$mib -o run -- python3 tools/time_lib.py $mib 10 > $O/kts.log 2>&1 || { tail -5 $O/kts.log; exit 1; }
  echo "$mib MiB $(python3 tools/kt_sum.py $O/kts_$mib | tr -d '\n ' | sed 's/.*"ms_span"/"ms_span"/')"
done
