# A/B: build/ab/*.so alternately (same box, 2 rounds), then the occupancy
# sensitivity of the first one (LDS pad: 3 -> 2 workgroups per CU)
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for L in build/ab/*.so; do
    HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/time_lib.py 1024 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
L=$(ls build/ab/*.so | head -1)
HH_LDS_PAD_KIB=12 HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 120 python tools/time_lib.py 1024 5 2>&1 | grep -v amdgpu.ids | sed 's/^/pad12 /'
