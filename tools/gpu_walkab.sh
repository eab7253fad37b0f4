# Same-box A/B of library variants and k_front walk bounds on the 1 GiB
# kjv-tiled stream.  Usage: bash tools/gpu_walkab.sh LIB[:FWALK] ...
# (LIB "-" = the in-tree build; FWALK sets HH_FRONT_WALK).  Two rounds,
# interleaved, each variant in its own process.
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
    lib=${v%%:*}; fw=${v#*:}; [ "$fw" = "$v" ] && fw=
    [ "$lib" = "-" ] && lib=$GRAFT_REPO_ROOT/huffmandecoderongpus_amd/libhiphuff.so
    echo "variant $v"
    HIPHUFF_LIB=$lib HH_FRONT_WALK=$fw timeout -k 10 180 python3 tools/time_lib.py ${MIB:-1024} 7 $SRC 2>>gpurun_out/ab.err || exit 1
  done
done
