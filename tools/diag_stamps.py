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

NAMES = ["counter+stage-load", "lookback(A)", "emit-setup(A)", "decode(B)+emit(A)", "walk(B)", "table(B)"]
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
cyc = raw[:, :6].astype(np.float64)
rounds = int((raw[:, 6] & 0xffffffff).sum()); slow = int((raw[:, 6] >> 32).sum()); spins = int(raw[:, 7].sum())
ntiles = (syn.bits + 255 * 288 - 1) // (255 * 288)
tot = cyc.sum(0)
print(f"ms={st['ms_total']:.3f} blocks={len(cyc)} tiles={ntiles} ok={n == syn.decoded_bytes}")
per_block = cyc.sum(1)
print(f"cycles per block: mean {per_block.mean():.0f} max {per_block.max():.0f} -> "
      f"{per_block.mean() / (st['ms_total'] * 1e-3) / 1e9:.2f} GHz implied")
for i, nm in enumerate(NAMES):
    print(f"{nm:12s} {tot[i] / ntiles:10.0f} cycles/tile  {100 * tot[i] / tot.sum():5.1f}%")
print(f"look-back: {rounds / ntiles:.2f} rounds/tile, {spins / ntiles:.2f} spins/tile, "
      f"{slow} serial-path tiles of {ntiles}")
sp = max(spins, 1)
print(f"per spin: nearest missing lane {raw[:, 8].sum() / sp:.1f}, farthest {raw[:, 9].sum() / sp:.1f}, "
      f"granule missing in {100 * raw[:, 10].sum() / sp:.0f}% of spins, first INCL lane {raw[:, 11].sum() / sp:.1f}")

tt = dec.tile_times()[:ntiles].astype(np.int64)
if len(tt):
    grab, pub, lb0, lb1, blk = tt[:, 0], tt[:, 1], tt[:, 2], tt[:, 3], tt[:, 4]
    t0 = grab[grab > 0].min()
    ok = (lb0 > 0) & (lb1 > 0)
    wait = (lb1 - lb0)[ok] * 10.0 / 1000      # us (100 MHz)
    print(f"look-back wait us: mean {wait.mean():.2f} p50 {np.median(wait):.2f} p90 {np.percentile(wait, 90):.2f} max {wait.max():.2f}")
    # lateness: latest granule among the 8 predecessors, relative to look-back start
    idx = np.arange(len(tt))
    late = np.full(len(tt), -1e9)
    for k in range(1, 9):
        j = idx - k
        m = j >= 0
        late[m] = np.maximum(late[m], (pub[j[m]] - lb0[m]) * 0.01)
    late_ok = late[ok]
    print(f"latest of 8 predecessors' granules after look-back start, us: mean {late_ok.mean():.2f} "
          f"p50 {np.median(late_ok):.2f} p90 {np.percentile(late_ok, 90):.2f}")
    w_minus_late = wait - np.maximum(late_ok, 0)
    print(f"wait minus that lateness, us: mean {w_minus_late.mean():.2f} p50 {np.median(w_minus_late):.2f}")
    it = (pub - grab) * 0.01
    print(f"grab->publish (one iteration + wait) us: mean {it.mean():.2f} p50 {np.median(it):.2f}")
    # per-block iteration period
    order = np.lexsort((grab, blk))
    b2, g2 = blk[order], grab[order]
    same = b2[1:] == b2[:-1]
    per = (g2[1:] - g2[:-1])[same] * 0.01
    print(f"iteration period per block us: mean {per.mean():.2f} p50 {np.median(per):.2f} p90 {np.percentile(per, 90):.2f}")
    # how far apart in grab time are consecutive tiles
    dg = (grab[1:] - grab[:-1]) * 0.01
    print(f"grab(t) - grab(t-1) us: mean {dg.mean():.3f} p1 {np.percentile(dg, 1):.2f} p99 {np.percentile(dg, 99):.2f}")
    np.save(os.path.join(ROOT, "gpurun_out", "tile_times.npy"), tt)
