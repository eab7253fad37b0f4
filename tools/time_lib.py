"""A/B timing: k_decode on the 1 GiB synthetic stream with the library named
by HIPHUFF_LIB (default: the in-tree build); prints the median of N runs."""
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
hf, text = synth.load_source(os.path.join(ROOT, "files"))
syn = synth.tiled_stream(hf, text, mib << 20)
dec = H.Decoder(0)
dec.set_tree(syn.tree)
out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
ms = []
for _ in range(reps + 1):
    n = dec.decode_device(syn.data, syn.bits, out)
    ms.append(dec.stats()["ms_total"])
ok = n == syn.decoded_bytes and synth.verify_tiled(out, syn)
print(f"{os.path.basename(os.environ.get('HIPHUFF_LIB', 'libhiphuff.so'))}: median {statistics.median(ms[1:]):.3f} ms "
      f"min {min(ms[1:]):.3f} ok={ok}", flush=True)
