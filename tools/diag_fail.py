"""Diagnostic: decode each fixture on the GPU and report the first failed
walk (tile, lane, exit, count, tile end), if any."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402

L = H.lib()
L.hh_debug_failure.restype = C.c_int
for name in sys.argv[1:] or ["paper1", "news", "book2", "kjv.txt", "E.coli"]:
    hf = H.HuffFile.load(os.path.join(ROOT, "files", name + ".huff"))
    dec = H.Decoder(0)
    dec.set_tree(hf.tree())
    out = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
    f = (C.c_uint32 * 5)()
    r = L.hh_debug_failure(dec._h, f)
    print(name, "bits", hf.bits, "n", len(out), "fallback", dec.stats()["exact_fallback"],
          "fail" if r else "", list(f) if r else "", flush=True)
    dec.close()
