# Same-box A/B of environment settings on the 1 GiB kjv-tiled stream.
# Usage: bash tools/gpu_envab.sh "VAR=val ..." "VAR=val ..." ...  ("" = defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SRC=${SRC:-kjv.txt}
export HH_TEXT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/text_$SRC.npy
rm -f $HH_TEXT_CACHE
timeout -k 10 120 python3 tools/time_lib.py 1 1 $SRC 2>>gpurun_out/ab.err || exit 1
for round in 1 2; do
  for v in "$@"; do
    echo "env [$v]"
    env $v timeout -k 10 180 python3 tools/time_lib.py ${MIB:-1024} 7 $SRC 2>>gpurun_out/ab.err || exit 1
  done
done
