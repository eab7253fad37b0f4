# Round-4: count pass with 4 regions per lane (k_cntm) against k_cnt
# (HH_CNT_M=1): instruction mix, waits and the vector-memory path.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
A="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE"
B="TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "count_pass_regions or capacity" --timeout 120 --timeout-method thread > $O/t.log 2>&1; tail -3 $O/t.log
ROUNDS=2 timeout -k 10 300 bash tools/gpu_ab.sh "- HH_CNT_M=1" "- HH_CNT_M=2" "- HH_CNT_M=4" > $O/ab.log 2>&1; cat $O/ab.log
SRC=bytes ROUNDS=1 timeout -k 10 300 bash tools/gpu_ab.sh "- HH_CNT_M=1" "- HH_CNT_M=2" "- HH_CNT_M=4" > $O/abb.log 2>&1; cat $O/abb.log
for m in ${MS:-2 4}; do
  for p in A B; do
    C=${!p}
    HH_CNT_M=$m timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/pmc_m${m}_$p -o run -- python3 tools/time_lib.py 1024 3 > $O/pmc_m${m}_$p.log 2>&1 || { tail -5 $O/pmc_m${m}_$p.log; exit 1; }
  done
  python3 tools/pmc_quick.py $O/pmc_m${m}_A > $O/pmc_m${m}_A.json && python3 tools/pmc_quick.py $O/pmc_m${m}_B > $O/pmc_m${m}_B.json
  echo "== M=$m"; python3 -c "
import json,sys
for p in 'AB':
    d=json.load(open('$O/pmc_m${m}_'+p+'.json'))
    for k in ('k_cnt','k_cntm'):
        if k in d: print(p,k,json.dumps({a:(round(b) if b>100 else b) for a,b in d[k].items()}))
"
done
