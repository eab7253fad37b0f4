set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/libhiphuff_stamps.so timeout -k 10 200 python tools/diag_stamps.py ${1:-1024} > gpurun_out/stamps.log 2>&1; rc=$?; cat gpurun_out/stamps.log; exit $rc
