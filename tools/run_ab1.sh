set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/diag_fixture.py hello paper1 news book2 kjv.txt E.coli > gpurun_out/d1.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not eight_shards and not hufx and not 2_31" > gpurun_out/t.log 2>&1 || exit 1
RUNS=5 bash tools/ab.sh build/libhiphuff_head.so build/libhiphuff_new.so > gpurun_out/ab.log || exit 1
SRC=E.coli RUNS=5 bash tools/ab.sh build/libhiphuff_head.so build/libhiphuff_new.so > gpurun_out/ab_ecoli.log || exit 1
export HH_TEXT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/text_kjv.txt.npy
timeout -k 10 120 python3 tools/time_lib.py 1 1 kjv.txt 2>>gpurun_out/ab.err || exit 1
HIPHUFF_LIB=build/libhiphuff_diag.so HH_DIAG=1 timeout -k 10 180 python3 tools/time_lib.py 1024 3 kjv.txt > gpurun_out/diag.log 2>>gpurun_out/ab.err || exit 1
