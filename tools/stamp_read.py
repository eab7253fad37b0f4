"""Phase stamps of the two passes' first workgroups (the HH_XP_STAMP
experiment build, kept out of the product source: git apply
tools/xp_stamp.patch && bash tools/mkvar.sh stamp -DHH_XP_STAMP && git
checkout huffmandecoderongpus_amd/csrc/hh_fsm.hip; run with
HIPHUFF_LIB=build/var/stamp.so HIPHUFF_AB_BUILD=1): s_memrealtime (100 MHz)
in wave 0 of k_cntm's and k_emf's first main workgroup, for the kjv-tiled
stream at a few sizes -- where a decode's fixed cost goes.

    python tools/stamp_read.py
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

cache = os.environ.get("HH_TEXT_CACHE")
hf = H.HuffFile.load(os.path.join(ROOT, "files", "kjv.txt.huff"))
text = np.load(cache)
for kib in (256, 65536, 1048576):
    syn = synth.tiled_stream(hf, text, kib << 10)
    out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
    dec = H.Decoder(0)
    dec.set_tree(syn.tree)
    buf = np.zeros(16, np.uint64)
    rows = []
    for _ in range(3):
        n = dec.decode_device(syn.data, syn.bits, out)
        torch.cuda.synchronize()
        H.lib().hh_debug_counters(dec._h, buf.ctypes.data)
        c = [int(v) for v in buf]
        us = lambda a, b: round((c[b] - c[a]) * 0.01, 2)   # noqa: E731
        rows.append({"count": {"fill": us(0, 1), "first_loads": us(1, 2), "first_counts": us(2, 3),
                               "first_walks_stores": us(3, 4), "rest": us(4, 5), "wg_total": us(0, 5)},
                     "gap_count_wg_end_to_emit_wg_start": us(5, 8),
                     "emit": {"fill_and_mx": us(8, 9), "first_loads": us(9, 10), "first_emission": us(10, 11),
                              "first_copyout": us(11, 12), "rest": us(12, 13), "wg_total": us(8, 13)},
                     "ms_total": round(dec.stats()["ms_total"], 4), "ok": n == syn.decoded_bytes})
    dec.close()
    print(json.dumps({"KiB": kib, "runs": rows[1:]}), flush=True)
    del out, syn
    torch.cuda.empty_cache()
