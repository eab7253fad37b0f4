"""evaluate()-scope timing of hh_decode_host on the tiled kjv stream:
python3 tools/time_eval.py [MiB] [reps].  HH_HOST_SERIAL=1 selects the
unpipelined path, HH_PIPE_CHUNK_KB the chunk size."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import huffmandecoderongpus_amd as H  # noqa: E402
from huffmandecoderongpus_amd import synth  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
files = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "files")
hf, text = synth.load_source(files, "kjv.txt")
syn = synth.tiled_stream(hf, text, mib << 20)
host = syn.data[: syn.compressed_bytes].cpu().numpy()
t0 = time.perf_counter()
r = bench.evaluate_scope(H, hf, host, syn.bits, syn.decoded_bytes, reps,
                         lambda o: synth.verify_tiled(torch.from_numpy(o).cuda(), syn))
r["wall_s"] = round(time.perf_counter() - t0, 2)
r["env"] = {k: os.environ[k] for k in ("HH_HOST_SERIAL", "HH_PIPE_CHUNK_KB") if k in os.environ}
print(r, flush=True)
