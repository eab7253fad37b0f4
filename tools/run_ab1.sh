set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export HH_TEXT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/text_kjv.txt.npy
rm -f $HH_TEXT_CACHE
timeout -k 10 120 python3 tools/time_lib.py 1 1 kjv.txt 2>>gpurun_out/ab.err || exit 1
HH_FLAGS=2 timeout -k 10 300 python3 tools/time_lib.py 1024 3 kjv.txt > gpurun_out/seg.log 2>>gpurun_out/ab.err || exit 1
