"""Diagnostic (GPU): the state-machine path on a fixture against the host
emulator (tests/emu) -- count-pass arrays tile by tile, then the output
against the oracle.  python tools/diag_fsm.py [fixture]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from oracle import oracle as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "kjv.txt"
hf = H.HuffFile.load(os.path.join(ROOT, "files", name + ".huff"))
ref = O.OracleHuff.load(os.path.join(ROOT, "files", name + ".huff")).chain_decode()
E = C.CDLL(os.path.join(ROOT, "tests", "emu", "libhh_emu.so"))
E.hh_fsm_emu_decode.restype = C.c_int64
E.hh_fsm_emu_decode.argtypes = [C.c_void_p] * 3 + [C.c_int32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_int32,
                                                   C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint64,
                                                   C.c_void_p, C.c_void_p, C.c_void_p]
E.hh_fsm_emu_arrays.restype = C.c_int64
E.hh_fsm_emu_arrays.argtypes = [C.c_void_p] * 4
iz = np.ascontiguousarray(hf.izero, np.int32)
io = np.ascontiguousarray(hf.ione, np.int32)
sy = np.ascontiguousarray(hf.sym, np.uint8)
d = np.zeros((hf.bits + 7) // 8 + 64, np.uint8)
d[: (hf.bits + 7) // 8] = np.asarray(hf.payload, np.uint8)[: (hf.bits + 7) // 8]
eout = np.zeros(hf.bits + 16, np.uint8)
st = np.zeros(9, np.int64)
n_e = E.hh_fsm_emu_decode(iz.ctypes.data, io.ctypes.data, sy.ctypes.data, len(iz), d.ctypes.data, hf.bits, 0, -1,
                          0, 0, 0, eout.ctypes.data, len(eout), st.ctypes.data, None, None)
S = int(st[3])
nt = (hf.bits + 64 * S - 1) // (64 * S)
erec = np.zeros(nt * 64, np.uint32); efx = np.zeros((nt + 1) * 8, np.uint32)
ets = np.zeros(nt, np.int32); exs = np.zeros(nt, np.uint32)
E.hh_fsm_emu_arrays(erec.ctypes.data, efx.ctypes.data, ets.ctypes.data, exs.ctypes.data)
print(f"emu: n={n_e} ok={n_e == len(ref) and np.array_equal(eout[:n_e], ref)} S={S} G={st[4]} tiles={nt}")

dec = H.Decoder(0)
dec.set_tree(hf.tree())
pad = np.zeros(((hf.data.size + 64 + 3) // 4) * 4, dtype=np.uint8)
pad[: hf.data.size] = hf.data
data = torch.from_numpy(pad).to("cuda")
out = torch.zeros(hf.uncompressedsize + 4096, dtype=torch.uint8, device="cuda")
try:
    n = dec.decode_device(data, hf.bits, out)
except H.HipHuffError as e:
    n = -1
    print("decode error", e)
torch.cuda.synchronize()
print("stats", dec.stats())
grec = np.zeros(nt * 64, np.uint32); gfx = np.zeros((nt + 1) * 8, np.uint32)
gts = np.zeros(nt, np.int32); gxs = np.zeros(nt, np.uint32)
rc = H.lib().hh_debug_fsm(dec._h, nt, grec.ctypes.data, gfx.ctypes.data, gts.ctypes.data, gxs.ctypes.data)
print("debug rc", rc)
for nm, a, b in (("rec", grec, erec), ("fx", gfx[: nt * 8], efx[: nt * 8]), ("tsum", gts, ets), ("xs", gxs, exs)):
    bad = np.nonzero(a != b)[0]
    print(f"{nm}: {bad.size} differ" + (f"; first at {bad[0]}: gpu {a[bad[0]]:#x} emu {b[bad[0]]:#x}" if bad.size else ""))
    if nm == "rec" and bad.size:
        t, j = divmod(int(bad[0]), 64)
        print("  tile", t, "region", j, "gpu ent/cnt", a[bad[0]] & 255, a[bad[0]] >> 8, "emu", b[bad[0]] & 255, b[bad[0]] >> 8)
        print("  gpu rec tile:", [(int(x & 255), int(x >> 8)) for x in a[t * 64: t * 64 + 8]])
        print("  emu rec tile:", [(int(x & 255), int(x >> 8)) for x in b[t * 64: t * 64 + 8]])
got = out[: max(n, 0)].cpu().numpy()
m = min(len(got), len(ref))
bad = np.nonzero(got[:m] != ref[:m])[0]
print(f"gpu n={n} ref={len(ref)} mismatches={bad.size}" + (f" first at {bad[0]}" if bad.size else ""))
if bad.size:
    i = int(bad[0])
    print("  gpu", got[i - 8: i + 8].tolist())
    print("  ref", ref[i - 8: i + 8].tolist())
