"""Diagnostic: decode the synthetic kjv-tiled stream at several sizes, check
it against the tiled text on the GPU and report mismatches together with the
per-tile bases recorded by the kernel (HH_DEBUG_TILES)."""
import ctypes as C
import os
import sys

os.environ["HH_DEBUG_TILES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

L = H.lib()
L.hh_debug_tiles.restype = C.c_int
L.hh_debug_tiles.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
hf, text = synth.load_source(os.path.join(ROOT, "files"))
for mib in [int(a) for a in sys.argv[1:]] or [64, 256, 1024]:
    syn = synth.tiled_stream(hf, text, mib << 20)
    dec = H.Decoder(0)
    dec.set_tree(syn.tree)
    out = torch.zeros(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
    for rep in range(3):
        out.zero_()
        n = dec.decode_device(syn.data, syn.bits, out)
        torch.cuda.synchronize()
        Lt = syn.text.numel()
        exp = syn.text.repeat(syn.copies + 1)[: syn.decoded_bytes]
        bad = torch.nonzero(out[: syn.decoded_bytes] != exp).flatten()
        nt = (syn.bits + 512 * 256 - 1) // (512 * 256)
        buf = np.zeros((nt, 8), np.uint64)
        got_t = L.hh_debug_tiles(dec._h, buf.ctypes.data, nt)
        base = buf[:, 0].astype(np.int64)
        size = (buf[:, 1] & 0xffffffff).astype(np.int64)
        incons = np.nonzero(base[1:] != base[:-1] + size[:-1])[0]
        print(f"{mib} MiB rep {rep}: n {n} want {syn.decoded_bytes} mismatches {bad.numel()} "
              f"tiles {got_t} inconsistent {len(incons)} ms {dec.stats()['ms_total']:.3f}", flush=True)
        if bad.numel():
            b = bad[:4].tolist()
            tt = np.searchsorted(base, b[0], side="right") - 1
            print("   first", b, "tile", tt, "base", base[tt], "size", size[tt],
                  "state", hex(int(buf[tt, 1]) >> 32), "excl", int(buf[tt, 2]), flush=True)
        cnt = ((buf[:, 3] & 0xfffff).astype(np.int64) ^ 0x80000) - 0x80000
        excl = buf[:, 2].astype(np.int64)
        bad_excl = np.nonzero(excl[1:] != excl[:-1] + cnt[:-1])[0]
        print("   excl chain breaks:", len(bad_excl), bad_excl[:10].tolist(), flush=True)
        for i in bad_excl[:4]:
            print(f"   tile {i}: excl {excl[i]} cnt {cnt[i]} -> next excl {excl[i+1]} (diff {excl[i+1]-excl[i]-cnt[i]})"
                  f" state {hex(int(buf[i, 1]) >> 32)} tab {hex(int(buf[i, 3]))}", flush=True)
            for q in (i, i + 1):
                u = int(buf[q, 4])
                print(f"      tile {q} look-back: incl tile {u} value {int(buf[q, 5])} (true {excl[u] + cnt[u] if 0 <= u < nt else '-'})"
                      f" summed {int(buf[q, 6])} (true {excl[q] - (excl[u] + cnt[u]) if 0 <= u < nt else '-'}) rounds {int(buf[q, 7])}", flush=True)
        for i in incons[:5]:
            print("   incons tile", i, "base", base[i], "size", size[i], "next base", base[i + 1],
                  "state", hex(int(buf[i, 1]) >> 32), hex(int(buf[i + 1, 1]) >> 32), flush=True)
    dec.close()
