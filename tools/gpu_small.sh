# The fixed cost per decode: the 64 and 128 MiB
# kjv-tiled decodes under a kernel trace (plain decoder, bench.py: kernel
# durations and the gaps between launches, tools/kt_sum.py), then the count
# pass's regions per lane (HH_CNT_M 1, 2, 4) A/B at both sizes.
# Output under gpurun_out/small.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/small
mkdir -p $O
for mib in 64 128; do
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt$mib -o run -- python3 bench.py --size-mib $mib --steps 20 --no-extra --no-cpu-baseline > $O/bench$mib.json 2> $O/kt$mib.err || { tail -5 $O/kt$mib.err; exit 1; }
    python3 tools/kt_sum.py $O/kt$mib > $O/kt$mib.sum.json || exit 1
    cat $O/kt$mib.sum.json
done
for mib in 64 128; do
    MIB=$mib ROUNDS=2 bash tools/gpu_ab.sh "- HH_CNT_M=2" "- HH_CNT_M=1" "- HH_CNT_M=4" > $O/ab_m$mib.log 2>&1 || { tail -5 $O/ab_m$mib.log; exit 1; }
    cat $O/ab_m$mib.log
done
echo done
