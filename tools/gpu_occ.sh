cd $GRAFT_REPO_ROOT
for pad in 0 12 40; do
  HH_LDS_PAD_KIB=$pad HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/ab/G.so timeout -k 10 120 python tools/time_lib.py 1024 5 2>&1 | grep -v amdgpu.ids | sed "s/^/pad $pad KiB: /" || exit 1
done
