# A/B timing of decoder settings on the 1 GiB kjv stream, alternated:
# AB="ENV=a ENV=b" (an empty entry: the default).  Every step under its own limit.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${AB:-_}; do
    [ "$v" = "_" ] && v=""
    env $v timeout -k 10 120 python3 tools/time_lib.py ${MIB:-1024} 5 ${SRC:-kjv.txt} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$v $(grep '{' gpurun_out/ab.log)"
  done
done
