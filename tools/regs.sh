#!/bin/bash
# Register / spill / occupancy summary of the kernels in one .hip file
# (hipcc's kernel-resource-usage remarks), filtered by a name pattern.
#   tools/regs.sh huffmandecoderongpus_amd/csrc/hh_fsm.hip 'k_cnt|k_emf' [extra hipcc flags]
f=$1; pat=${2:-.}; shift 2
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Ihuffmandecoderongpus_amd/csrc "$@" -c "$f" -o /tmp/regs_$$.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
pat = re.compile(sys.argv[1]); cur = None; rows = []
keys = {"VGPRs": "vgpr", "TotalSGPRs": "sgpr", "Occupancy [waves/SIMD]": "occ", "SGPRs Spill": "sspill",
        "VGPRs Spill": "vspill", "ScratchSize [bytes/lane]": "scratch"}
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|TotalSGPRs|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|ScratchSize \[bytes/lane\]): (\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k == "Function Name": cur = {"name": v}; rows.append(cur)
    elif cur is not None: cur[keys[k]] = v
for r in rows:
    if pat.search(r["name"]):
        print("%-62s" % r["name"][:62], " ".join("%s %s" % (k, r.get(k)) for k in ("vgpr", "sgpr", "occ", "vspill", "sspill", "scratch")))
' "$pat"
rm -f /tmp/regs_$$.o
