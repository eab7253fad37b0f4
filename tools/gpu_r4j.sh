# evaluate() scope A/B: the session-start build against the current one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
export HH_TEXT_CACHE=$O/text_kjv.txt.npy
[ -f $HH_TEXT_CACHE ] || timeout -k 10 120 python3 tools/time_lib.py 1 1 kjv.txt 2>>$O/ab.err
for r in 1 2; do
  for L in build/var/start.so huffmandecoderongpus_amd/libhiphuff.so; do
    HIPHUFF_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 tools/time_eval.py 1024 5 || exit 1
  done
done
