"""Decode the tiled synthetic stream of a fixture at several sizes with the
library HIPHUFF_LIB names (default: the in-tree build) and report errors or
the first mismatching byte (and its 32-bit word of the tiled text).

    python tools/diag_tiled.py kjv.txt 64 256 1024
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

src = sys.argv[1]
hf, text = synth.load_source(os.path.join(ROOT, "files"), src)
for mib in map(int, sys.argv[2:]):
    syn = synth.tiled_stream(hf, text, mib << 20)
    dec = H.Decoder(0)
    dec.set_tree(syn.tree)
    out = torch.zeros(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
    try:
        n = dec.decode_device(syn.data, syn.bits, out)
    except H.HipHuffError as e:
        print(src, mib, "error", e, flush=True)
        import ctypes as C
        f = (C.c_uint32 * 5)()
        H.lib().hh_debug_failure.argtypes = [C.c_void_p, C.c_void_p]
        print("  debug", H.lib().hh_debug_failure(dec._h, f), list(f), "ntiles", syn.bits // dec.tile_bits(), flush=True)
        continue
    torch.cuda.synchronize()
    ok = synth.verify_tiled(out, syn)
    first = -1
    if not ok:                                   # the first bad byte, 256 MiB at a time
        L = syn.text.numel()
        for c0 in range(0, syn.decoded_bytes, 1 << 28):
            c1 = min(c0 + (1 << 28), syn.decoded_bytes)
            idx = torch.arange(c0, c1, device="cuda") % L
            bad = torch.nonzero(out[c0:c1] != syn.text[idx]).flatten()
            if bad.numel():
                first = c0 + int(bad[0])
                break
    print(src, mib, "n", n, "want", syn.decoded_bytes, "ok", ok, "first_bad", first,
          "tile_bits", dec.tile_bits(), "stats", dec.stats(), flush=True)
    dec.close()
    del out, want
