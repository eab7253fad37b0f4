set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/diag_tiled.py E.coli 1024 > gpurun_out/d1.log 2>&1 || exit 1
RUNS=5 bash tools/ab.sh build/libhiphuff_base.so build/libhiphuff_new.so build/libhiphuff_nt.so build/libhiphuff_minw4.so > gpurun_out/ab.log || exit 1
HH_TEXT_CACHE=gpurun_out/text_kjv.txt.npy HH_OVERLAP=0 timeout -k 10 180 python3 tools/time_lib.py 1024 5 kjv.txt >> gpurun_out/ab.log 2>>gpurun_out/ab.err || exit 1
for v in new nt; do
  HIPHUFF_LIB=build/libhiphuff_$v.so HH_TEXT_CACHE=gpurun_out/text_kjv.txt.npy timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw_$v -o run -- python3 tools/time_lib.py 1024 2 kjv.txt > gpurun_out/pw_$v.log 2>&1 || exit 1
done
SRC=E.coli RUNS=5 bash tools/ab.sh build/libhiphuff_base.so build/libhiphuff_new.so build/libhiphuff_nt.so build/libhiphuff_minw4.so > gpurun_out/ab_ecoli.log
HIPHUFF_LIB=build/libhiphuff_diag.so HH_DIAG=1 HH_TEXT_CACHE=gpurun_out/text_kjv.txt.npy timeout -k 10 180 python3 tools/time_lib.py 1024 3 kjv.txt > gpurun_out/diag.log 2>>gpurun_out/ab.err
