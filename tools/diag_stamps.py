"""Diagnostic only: per-phase cycles of the fused kernel (needs a library
built with `make lib HIPEXTRA=-DHH_STAMPS`)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

NAMES = ["top/counter", "stage", "region", "walk", "table", "count-lookback", "emit", "granule-wait"]
size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
hf, text = synth.load_source(os.path.join(ROOT, "files"))
syn = synth.tiled_stream(hf, text, size << 20)
dec = H.Decoder(0)
dec.set_tree(syn.tree)
out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
for _ in range(3):
    n = dec.decode_device(syn.data, syn.bits, out)
st = dec.stats()
cyc = dec.phase_cycles().astype(np.float64)
ntiles = (syn.bits + 255 * 288 - 1) // (255 * 288)
tot = cyc.sum(0)
print(f"ms={st['ms_total']:.3f} blocks={len(cyc)} tiles={ntiles} ok={n == syn.decoded_bytes}")
per_block = cyc.sum(1)
print(f"cycles per block: mean {per_block.mean():.0f} max {per_block.max():.0f} -> "
      f"{per_block.mean() / (st['ms_total'] * 1e-3) / 1e9:.2f} GHz implied")
for i, nm in enumerate(NAMES):
    print(f"{nm:12s} {tot[i] / ntiles:10.0f} cycles/tile  {100 * tot[i] / tot.sum():5.1f}%")
