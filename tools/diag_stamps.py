"""Diagnostic only: per-phase shader cycles of k_decode (needs the library
built with -DHH_STAMPS: `make stamps`, loaded via HIPHUFF_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

NAMES = ["stage", "pass1", "walks", "table", "entry+lookback", "scan", "pass2", "walk-wait"]
size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
hf, text = synth.load_source(os.path.join(ROOT, "files"))
syn = synth.tiled_stream(hf, text, size << 20)
dec = H.Decoder(0)
dec.set_tree(syn.tree)
out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
for _ in range(3):
    n = dec.decode_device(syn.data, syn.bits, out)
st = dec.stats()
raw = dec.phase_cycles()
cyc = raw[:, :len(NAMES)].astype(np.float64)
print(f"ms={st['ms_total']:.3f} blocks={len(cyc)} ok={n == syn.decoded_bytes and synth.verify_tiled(out, syn)}")
tot = cyc.sum(0)
for i, nm in enumerate(NAMES):
    print(f"  {nm:12s} {tot[i] / tot.sum() * 100:6.2f}%  mean/block {cyc[:, i].mean() / 2.4e6:8.3f} ms@2.4GHz")
ex = raw[:, 8:12].astype(np.float64).sum(0)
if ex[2]:
    print(f"  look-backs {ex[2]:.0f} (entering state + exclusive prefix) at {ex[1] / ex[2]:.0f} cyc each")
print(f"  total cycles/block mean {cyc.sum(1).mean():.3e} max {cyc.sum(1).max():.3e}")
