# Wave start/end spans of k_cntm and k_emf (a -DHH_WSPAN build, build/var/wspan.so)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in 1024 64; do
  HH_WSPAN_DUMP=$GRAFT_REPO_ROOT/gpurun_out/wspan HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/var/wspan.so HH_WSPAN=1 HH_NO_PHASES=1 timeout -k 10 120 python3 tools/time_lib.py $m 3 kjv.txt || exit 1
done
