# Round-4 GPU check: tests, same-box A/B of the previous commit against the
# working tree (and 384-bit regions), LDS counters of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -3 $O/t.log
ROUNDS=2 timeout -k 10 400 bash tools/gpu_ab.sh base - "- HH_LANE_BITS=384" > $O/ab.log 2>&1; cat $O/ab.log
for v in base cur; do
  L=$GRAFT_REPO_ROOT/build/var/$v.so; [ $v = cur ] && L=$GRAFT_REPO_ROOT/huffmandecoderongpus_amd/libhiphuff.so
  HIPHUFF_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d $O/pmc_$v -o run -- python3 tools/time_lib.py 1024 3 > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  python3 tools/pmc_quick.py $O/pmc_$v > $O/pmc_$v.json; echo "== $v"; cat $O/pmc_$v.json
done
