# rocprofv3 kernel stats and counters (tools/profile.sh) for bench.py's
# secondary workloads, each summarised into profiles/<tag>_<name>_kernels.json
# (tools/prof_summary.py; pmc_latest.json stays the headline's).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05}
E=gpurun_out/evidence
mkdir -p $E
one() {   # name, source, flags, workload label
  echo "[$(date +%T)] $1"
  SRC=$2 HH_FLAGS=$3 bash tools/profile.sh ${TAG}_$1 > $E/profile_$1.log 2>&1 || { tail -20 $E/profile_$1.log; exit 1; }
  python3 tools/prof_summary.py ${TAG}_$1 "$4" > $E/prof_summary_$1.log 2>&1 || { tail -20 $E/prof_summary_$1.log; exit 1; }
  cp profiles/${TAG}_$1_kernels.json profiles/${TAG}_$1_kernel_stats.csv $E/
}
one ecoli_sm E.coli 4 "synthetic 1024 MiB E.coli-tiled .huff, general pipeline (HH_FLAG_NO_FIXED)"
one iid iid 0 "synthetic 1024 MiB i.i.d. kjv-unigram .huff (splitmix64 seed 0x5eed5eed)"
one bytes bytes 0 "synthetic 1024 MiB byte-alphabet .huff (256-symbol Huffman code, Zipf s=1.1)"
echo "[$(date +%T)] done"
