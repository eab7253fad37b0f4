# A/B: time build/ab/*.so alternately (same box), 2 rounds
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for L in build/ab/*.so; do
    HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/time_lib.py 1024 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
