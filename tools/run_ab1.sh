set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RUNS=5 bash tools/ab.sh build/libhiphuff_new.so build/libhiphuff_ew8.so build/libhiphuff_ew2.so > gpurun_out/ab.log || exit 1
SRC=E.coli RUNS=5 bash tools/ab.sh build/libhiphuff_new.so build/libhiphuff_ew8.so build/libhiphuff_ew2.so > gpurun_out/ab_ecoli.log || exit 1
export HH_TEXT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/text_kjv.txt.npy
timeout -k 10 120 python3 tools/time_lib.py 1 1 kjv.txt 2>>gpurun_out/ab.err || exit 1
