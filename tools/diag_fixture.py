"""Decode each fixture on the GPU with the library HIPHUFF_LIB names (default:
the in-tree build) and report the first mismatching byte against the oracle.

    python tools/diag_fixture.py paper1 news ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from oracle import oracle as O  # noqa: E402

for name in sys.argv[1:]:
    path = os.path.join(ROOT, "files", name + ".huff")
    hf = H.HuffFile.load(path)
    want = O.OracleHuff.load(path).chain_decode()
    dec = H.Decoder(0)
    dec.set_tree(hf.tree())
    got = dec.decode_host(hf.payload, hf.bits, len(want) + 4096)
    st = dec.stats()
    n = min(len(got), len(want))
    bad = np.nonzero(got[:n] != want[:n])[0]
    first = int(bad[0]) if len(bad) else -1
    print(name, "len", len(got), "want", len(want), "first_bad", first, "nbad", len(bad),
          "tile_bits", dec.tile_bits(), "fallback", st["exact_fallback"], flush=True)
    if first >= 0:
        print("  got ", bytes(got[first:first + 24]), "\n  want", bytes(want[first:first + 24]))
    dec.close()
