"""Counters of the single pass (k_one) from its diagnostic build
(make variant V=odbg HIPEXTRA=-DHH_ONE_DBG; run with
HIPHUFF_LIB=build/libhiphuff_odbg.so HH_ONE_DBG=1): per decode of the
kjv-tiled stream, the tiles, look-back polls and restarts, fix rounds,
lane-0 redos, overflowing tiles, block-map spins and the wave cycles of each
phase (s_memtime, summed over waves).

    python tools/one_diag.py [MiB]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

NAMES = ["tiles", "polls", "restarts", "fix_tiles", "fix_rounds", "redo0", "ovf", "ring_spins",
         "cyc_emit", "cyc_lookback", "cyc_out", "cyc_take", "cyc_all"]
mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
src = sys.argv[2] if len(sys.argv) > 2 else "kjv.txt"
hf0 = H.HuffFile.load(os.path.join(ROOT, "files", src + ".huff"))
d0 = H.Decoder(0, flags=H.FLAG_TWO_PASS)
d0.set_tree(hf0.tree())
text = d0.decode_host(hf0.payload, hf0.bits, hf0.uncompressedsize + 3)
d0.close()
syn = synth.tiled_stream(hf0, text, mib << 20)
out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
dec = H.Decoder(0, lane_bits=int(os.environ.get("HH_LANE_BITS", "0")))
dec.set_tree(syn.tree)
buf = np.zeros(16, np.uint64)
for i in range(3):
    n = dec.decode_device(syn.data, syn.bits, out)
    torch.cuda.synchronize()
    H.lib().hh_debug_counters(dec._h, buf.ctypes.data)
    c = {k: int(v) for k, v in zip(NAMES, buf)}
    ok = n == syn.decoded_bytes and synth.verify_tiled(out, syn)
    st = dec.stats()
    print(json.dumps({"mib": mib, "ok": bool(ok), "sm": st["state_machine"], "ms": round(st["ms_total"], 4), **c}), flush=True)
