"""Where does bench.py's evaluate() time differ from tools/time_eval.py's?
bench.evaluate_scope on the 1 GiB kjv-tiled stream: at the start of the
process, after the bench's device decodes of the same stream, and after the
small kjv.txt evaluate -- one JSON line per stage."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

dev = torch.device("cuda", 0)
hf, text = synth.load_source(os.path.join(ROOT, "files"), "kjv.txt", device=0)
syn = synth.tiled_stream(hf, text, 1024 << 20, device=dev)


def ev(tag):
    host = syn.data[: syn.compressed_bytes].cpu().numpy()
    r = bench.evaluate_scope(H, hf, host, syn.bits, syn.decoded_bytes, 5)
    print(json.dumps({"stage": tag, **r}), flush=True)


ev("fresh")
dec = H.Decoder(0)
dec.set_tree(syn.tree)
out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device=dev)
for _ in range(30):
    dec.decode_device_async(syn.data, syn.bits, out, torch.cuda.current_stream(dev))
dec.wait()
torch.cuda.synchronize()
ev("after device decodes")
r = bench.evaluate_scope(H, hf, hf.payload, hf.bits, hf.uncompressedsize, 20)
ev("after the kjv.txt evaluate")
del out
dec.close()
torch.cuda.empty_cache()
ev("after close + empty_cache")
