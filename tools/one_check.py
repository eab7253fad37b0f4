"""Single-pass decode check (hh_one.hip) on the GPU box: every fixture and the
kjv-tiled stream at the given sizes through the default path (the single
pass) and through HH_FLAG_TWO_PASS, byte-checked, with the device time.
One JSON line per case.

    python tools/one_check.py [MiB ...]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

sizes = [int(a) for a in sys.argv[1:]] or [64, 1024]
LB = int(os.environ.get("HH_LANE_BITS", "0"))      # region bits (0: the decoder's choice)
FIX = os.environ.get("ONE_FIXTURES", "1") != "0"
files = os.path.join(ROOT, "files")


def two_pass_text(name):
    """The fixture's text from the two-pass decoder (the reference for the single pass)."""
    import hashlib
    hf = H.HuffFile.load(os.path.join(files, name + ".huff"))
    dec = H.Decoder(0, flags=H.FLAG_TWO_PASS)
    dec.set_tree(hf.tree())
    text = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
    dec.close()
    if name == "kjv.txt":
        assert hashlib.sha256(text.tobytes()).hexdigest() == synth.KJV_SHA256
    return hf, text


def run(dec, data, bits, out, reps):
    n = dec.decode_device(data, bits, out)
    st = dec.stats()
    ts = []
    for _ in range(reps):
        dec.decode_device(data, bits, out)
        ts.append(dec.stats()["ms_total"])
    return n, st, (statistics.median(ts) if ts else st["ms_total"])


for name in ["hello", "paper1", "news", "book2", "world192.txt", "bible.txt", "kjv.txt", "E.coli"] if FIX else []:
    hf = H.HuffFile.load(os.path.join(files, name + ".huff"))
    if name in ("kjv.txt", "E.coli"):
        _, ref = two_pass_text(name)
    else:
        ref = np.fromfile(os.path.join(files, name), dtype=np.uint8)
    data = torch.from_numpy(np.concatenate([hf.payload, np.zeros(64, np.uint8)])).cuda()
    for flags in (H.FLAG_NO_FIXED, H.FLAG_NO_FIXED | H.FLAG_TWO_PASS):
        dec = H.Decoder(0, flags=flags)
        dec.set_tree(hf.tree())
        out = torch.zeros(hf.uncompressedsize + 4096, dtype=torch.uint8, device="cuda")
        n, st, ms = run(dec, data, hf.bits, out, 3)
        got = out[:n].cpu().numpy()
        ok = n == ref.size and np.array_equal(got, ref)
        bad = None
        if not ok and n == ref.size:
            d = np.nonzero(got != ref)[0]
            bad = [int(d[0]), int(d.size)]
        print(json.dumps({"case": name, "two": bool(flags & H.FLAG_TWO_PASS), "ok": ok, "n": int(n), "want": int(ref.size),
                          "sm": st["state_machine"], "ms": round(ms, 4), "first_bad": bad}), flush=True)
        dec.close()

hf, text = two_pass_text("kjv.txt")
for mib in sizes:
    syn = synth.tiled_stream(hf, text, mib << 20)
    out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
    for flags in (0, H.FLAG_TWO_PASS):
        dec = H.Decoder(0, lane_bits=LB, flags=flags)
        dec.set_tree(syn.tree)
        out.zero_()
        n, st, ms = run(dec, syn.data, syn.bits, out, 7)
        ok = n == syn.decoded_bytes and synth.verify_tiled(out, syn)
        frac = (syn.compressed_bytes + syn.decoded_bytes) / (ms * 1e-3) / 8e12
        print(json.dumps({"case": f"kjv-tiled {mib} MiB", "S": dec.tile_bits() // 64, "two": bool(flags), "ok": bool(ok), "n": int(n),
                          "sm": st["state_machine"], "ms": round(ms, 4), "frac": round(frac, 4)}), flush=True)
        dec.close()
