"""A/B timing (tools/ab.sh): the decode pipeline on the synthetic stream with
the library named by HIPHUFF_LIB (default: the in-tree build); prints one
JSON line with the median device time of each kernel phase over N runs and
whether the output matched the tiled text.

    python tools/time_lib.py [MiB] [runs] [source]   (source: kjv.txt | E.coli)
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
src = sys.argv[3] if len(sys.argv) > 3 else "kjv.txt"
hf, text = synth.load_source(os.path.join(ROOT, "files"), src)
syn = synth.tiled_stream(hf, text, mib << 20)
dec = H.Decoder(0)
dec.set_tree(syn.tree)
out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
ph = {"total": [], "sync": [], "scan": [], "emit": []}
ok = True
for i in range(reps + 1):
    n = dec.decode_device(syn.data, syn.bits, out)
    torch.cuda.synchronize()
    if i == 0:
        ok = n == syn.decoded_bytes and synth.verify_tiled(out, syn)
        continue
    st = dec.stats()
    for k in ph:
        ph[k].append(st["ms_" + k])
res = {"lib": os.path.basename(os.environ.get("HIPHUFF_LIB", H.LIB_PATH)), "mib": mib, "src": src,
       "ok": bool(ok), "fast": dec.stats()["exact_fallback"] == 0}
res.update({k: round(statistics.median(v), 4) for k, v in ph.items()})
print(json.dumps(res), flush=True)
