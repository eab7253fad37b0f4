set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export HH_TEXT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/text_kjv.npy
rm -f $HH_TEXT_CACHE
timeout -k 10 120 python3 tools/time_lib.py 1 1 kjv.txt 2>>gpurun_out/nolb.err || exit 1
for i in 1 2; do
echo "two-pass: $(HH_NO_PHASES=1 timeout -k 10 120 python3 tools/time_lib.py 1024 7 2>>gpurun_out/nolb.err)" || exit 1
echo "one nolb: $(HH_ONE=1 HH_NO_PHASES=1 HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/var/nolb.so HIPHUFF_AB_BUILD=1 timeout -k 10 120 python3 tools/time_lib.py 1024 7 2>>gpurun_out/nolb.err)" || exit 1
done
HH_ONE=1 HH_ONE_DBG=1 HIPHUFF_LIB=$GRAFT_REPO_ROOT/build/var/nolbd.so HIPHUFF_AB_BUILD=1 timeout -k 10 180 python3 tools/one_diag.py 1024 2>>gpurun_out/nolb.err || exit 1
echo done
