# Round-4: full GPU tests; kjv / bytes / E.coli phase split; kernel trace of
# production-like decodes (no phase events) at 64 MiB and 1 GiB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -3 $O/t.log
for src in kjv.txt bytes; do timeout -k 10 200 python3 tools/time_lib.py 1024 7 $src 2>>$O/ab.err; done
for mib in 64 1024; do
  HH_NO_PHASES=1 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$mib -o run -- python3 tools/time_lib.py $mib 20 > $O/kt_$mib.log 2>&1 || { tail -5 $O/kt_$mib.log; exit 1; }
  echo "== kernel trace $mib MiB"; python3 tools/kt_sum.py $O/kt_$mib | tr -d '\n '; echo
done
