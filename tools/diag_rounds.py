"""Diagnostic: decode fixtures with several LDS output-window sizes and
report mismatching segments against the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from oracle import oracle as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "kjv.txt"
kibs = [int(k) for k in sys.argv[2:]] or [8]
path = os.path.join(ROOT, "files", name + ".huff")
hf = H.HuffFile.load(path)
ref = O.OracleHuff.load(path).chain_decode()
for kib in kibs:
    os.environ["HH_OB_KIB"] = str(kib)
    for rep in range(2):
        dec = H.Decoder(0)
        dec.set_tree(hf.tree())
        d_in = torch.from_numpy(hf.data.copy()).cuda()
        d_out = torch.full((hf.uncompressedsize + 64,), 0xEE, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(d_in, hf.bits, d_out)
        torch.cuda.synchronize()
        got = d_out[:n].cpu().numpy()
        bad = got[: len(ref)] != ref[: len(got)]
        idx = np.nonzero(bad)[0]
        segs = []
        if len(idx):
            br = np.nonzero(np.diff(idx) > 1)[0]
            starts = np.concatenate([[idx[0]], idx[br + 1]])
            ends = np.concatenate([idx[br], [idx[-1]]]) + 1
            segs = list(zip(starts.tolist(), ends.tolist()))
        print(f"{name} {kib} KiB rep {rep}: mismatches {len(idx)} segments {len(segs)}", flush=True)
        for s, e in segs[:12]:
            v = got[s:e]
            print(f"   [{s},{e}) len {e - s}  uniq {np.unique(v)[:4].tolist()}  got {v[:6].tolist()} want {ref[s:s+6].tolist()}")
        dec.close()
