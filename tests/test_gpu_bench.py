"""bench.py's N > 1 path end to end on one GPU: two ranks
started by `bench.py --gpus 2` itself (torch.distributed.run), both on
cuda:0, over gloo (RCCL refuses two ranks on one GPU) -- the launcher,
init_process_group, the checked step, the timed full steps (decode, entry
exchange, any redo), the decode-only steps, the confirmation, the segments'
all-gather and the rank-reduced timing all run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_one_device(files_dir):
    from huffmandecoderongpus_amd import synth
    mib = 64
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--size-mib", str(mib), "--steps", "3",
           "--warmup", "1", "--backend", "gloo", "--one-device", "--no-cpu-baseline", "--no-extra"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    assert res["settle"]["confirmed_after_timed"] is True
    assert res["allgather"]["seams_ok"] is True
    hf, text = synth.load_source(files_dir, "kjv.txt")
    _, syms = synth.cut_bits(hf, text, 2 * (mib << 20))
    assert res["config"]["decoded_bytes"] == syms
    assert res["value"] > 0 and res["settle"]["decode_only"]["ms_per_step"] > 0
