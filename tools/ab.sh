# Same-box A/B of library variants: tools/ab.sh build/libA.so build/libB.so ...
# (each built in-tree beforehand, e.g. `make variant V=name HIPEXTRA=-DX=1`).
# Each variant runs in its own process, twice, interleaved, so clock drift
# between variants shows up as spread rather than as a difference.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MIB=${MIB:-1024}
RUNS=${RUNS:-7}
SRC=${SRC:-kjv.txt}
export HH_TEXT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/text_$SRC.npy
rm -f $HH_TEXT_CACHE
timeout -k 10 120 python3 tools/time_lib.py 1 1 $SRC 2>>gpurun_out/ab.err || exit 1
for round in 1 2; do
  for lib in "$@"; do
    HIPHUFF_LIB=$lib timeout -k 10 180 python3 tools/time_lib.py $MIB $RUNS $SRC 2>>gpurun_out/ab.err || exit 1
  done
done
