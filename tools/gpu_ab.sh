# Same-box A/B of library variants (tools/mkvar.sh) and environment settings
# on the 1 GiB kjv-tiled stream.  Each argument is "LIB [VAR=val ...]" (LIB
# "-": the in-tree build, else build/var/LIB.so).  ROUNDS rounds, interleaved,
# each variant in its own process under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SRC=${SRC:-kjv.txt}
export HH_TEXT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/text_$SRC.npy
rm -f $HH_TEXT_CACHE
timeout -k 10 120 python3 tools/time_lib.py 1 1 $SRC 2>>gpurun_out/ab.err || exit 1
VARS=("$@")
for round in $(seq ${ROUNDS:-2}); do
  for v in "${VARS[@]}"; do
    read -r lib envs <<< "$v"
    [ "$lib" = "-" ] && L=$GRAFT_REPO_ROOT/huffmandecoderongpus_amd/libhiphuff.so || L=$GRAFT_REPO_ROOT/build/var/$lib.so
    r=$(env HIPHUFF_LIB=$L HIPHUFF_AB_BUILD=1 $envs timeout -k 10 180 python3 tools/time_lib.py ${MIB:-1024} 7 $SRC 2>>gpurun_out/ab.err) || { echo "[$v] failed"; exit 1; }
    echo "[$v] $r"
  done
done
