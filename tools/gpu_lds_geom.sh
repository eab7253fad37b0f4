# The count step's LDS geometry: tools/ubench/ub_lds.hip
# (build/ub_lds) for each entry geometry at 16 waves per CU -- the time
# alone, then LDS instructions and bank-conflict cycles in a counter pass
# of its own.  Output under gpurun_out/lds_geom; tools/lds_geom_sum.py sums it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lds_geom
mkdir -p $O
for ent in 2 3 4 8; do
    timeout -k 10 60 build/ub_lds 2000 16 $ent | tee -a $O/times.txt || exit 1
    timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $O/e$ent -o run -- build/ub_lds 2000 16 $ent > $O/e$ent.log 2>&1 || { tail -5 $O/e$ent.log; exit 1; }
done
echo done
