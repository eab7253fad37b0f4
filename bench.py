#!/usr/bin/env python3
"""bench.py -- decoded MB/s and HBM roofline fraction of the HIP decoder.

Workload (BASELINE.json configs[2]): a synthetic 1 GiB English-text .huff --
kjv.txt tiled (about 349.4 copies) and encoded with the files/kjv.txt.huff
codebook, cut at a symbol boundary -- decoded on each MI355X.  One "step" is
one full decode of that stream with the input already resident in HBM:
hh_decode_device -- the state-machine decode (k_cntm: 128-bit heads, each
region's count and exit state in 8-bit steps of the count table, walks
where a guessed entering state was wrong; k_fscan1: tile bases, its last
block the block bases; k_emf: emission in 7-bit steps into LDS staging,
16-B copy-out) -- plus its
status readback.  For N > 1 the stream is N GiB, sharded
by whole tiles (weak scaling); each timed step is the rank's segment decode
(with its prologue tiles), queued asynchronously, no collective inside it --
the entry-state exchange (one 5-integer all-gather) runs on a checked step
before the timed region and once more after it (`settle`); the decoded
segments are all-gathered once after the timed region and reported
separately (`allgather`).

Prints ONE JSON line on rank 0.  `roofline.achieved` = (C + D algorithmic
bytes per decode) / the pipeline's average device time, measured with HIP
events on the launches' stream inside the timed region; `traffic` is the
HBM bytes per decode measured by rocprofv3 FETCH_SIZE/WRITE_SIZE passes
(profiles/pmc_latest.json, tools/profile.sh).  On one GPU the line also
carries `workloads` (the E.coli-tiled and i.i.d. kjv-unigram streams of the
same size) and `evaluate` (the reference's evaluate() scope:
host payload in, host symbols out).  `cpu_baseline` times the reference's
own linApproach (oracle/_ref, compiled from the reference's C sources) or,
if that was not built, the oracle's restatement, on a bounded sample
(kjv.txt.huff) on one host core.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size-mib", type=int, default=1024, help="compressed MiB per GPU")
    ap.add_argument("--files", default=os.path.join(ROOT, "files"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the E.coli / i.i.d. workloads and the evaluate()-scope timing")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="HBM traffic measured by rocprofv3 --pmc (tools/profile.sh)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo: tests)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (tests of the N > 1 path on a one-GPU box; gloo only)")
    return ap.parse_args()


def cpu_baseline(files_dir: str, seconds: float, name: str = "kjv.txt.huff") -> dict:
    """linApproach on files/<name>, one core: sweep jumpbits 1..14 once
    (the reference's testall sweep, mainrun.c:456-459), then repeat the best
    for ~`seconds`; report decoded MB/s of the median repeat."""
    from oracle import oracle as O
    path = os.path.join(files_dir, name)
    if O.ref_available():
        kind = "reference"
        h = O.RefHuff(path)
        run = lambda J: h.run("linApproach", J)          # noqa: E731
        D = h.uncompressedsize
    else:
        kind = "port"
        h = O.OracleHuff.load(path)
        run = h.lin_decode                                 # noqa: E731
        D = h.uncompressedsize
    best_j, best_t = None, None
    for J in range(1, 15):
        t0 = time.perf_counter()
        run(J)
        t = time.perf_counter() - t0
        if best_t is None or t < best_t:
            best_j, best_t = J, t
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        run(best_j)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    cpu = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(D / med / 1e6, 2), "unit": "MB/s", "cores": 1, "kind": kind, "jumpbits": best_j,
            "sample": (f"linApproach(jumpbits={best_j}) on files/{name} "
                       f"({D} B decoded), median of {len(times)} runs over ~{seconds:.0f} s, "
                       f"tables built inside each timed call; host {cpu}, "
                       f"nproc {os.cpu_count()}")}


_CPU_CHILD = """
import sys, time
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
h = O.RefHuff(sys.argv[2])
t0 = float(sys.argv[5])
while time.time() < t0:        # (every process loaded: all start together)
    time.sleep(0.001)
for _ in range(int(sys.argv[4])):
    h.run("linApproach", int(sys.argv[3]))
print(time.time(), flush=True)
"""


def cpu_baseline_tiled(H, hf, text, mib: int, jumpbits: int, reps: int, procs: int) -> dict:
    """The reference's linApproach (oracle/_ref) on the headline stream's
    shape at the largest size its HUFF header holds (int32 bits: 128 MiB of
    the kjv-tiled stream, saved as a .huff), jumpbits from the kjv.txt sweep:
    (a) one core, `reps` repeats, median; (b) `procs` processes on the host's
    cores at once, each decoding the whole stream twice -- the aggregate rate
    of independent decodes, the most a host running the reference's serial
    decoder on many streams gets."""
    import subprocess
    import tempfile
    import numpy as np
    from oracle import oracle as O
    from huffmandecoderongpus_amd import synth
    syn = synth.tiled_stream(hf, text, mib << 20, device="cpu")
    nb = (syn.bits + 7) // 8
    data = np.zeros(nb + H.PAYLOAD_PAD, np.uint8)
    data[:nb] = syn.data[:nb].numpy()
    D = syn.decoded_bytes
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, f"kjv_tiled_{mib}MiB.huff")
        H.HuffFile(hf.izero, hf.ione, hf.sym, syn.bits, D, data).save(path)
        del data, syn
        h = O.RefHuff(path)
        out = h.run("linApproach", jumpbits)
        ok = out.size == D and np.array_equal(out[: text.size], text)
        del out
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            h.run("linApproach", jumpbits)
            ts.append(time.perf_counter() - t0)
        del h
        t_go = time.time() + 5.0 + 0.2 * procs
        ps = [subprocess.Popen([sys.executable, "-c", _CPU_CHILD, ROOT, path, str(jumpbits), "2", repr(t_go)],
                               stdout=subprocess.PIPE, text=True) for _ in range(procs)]
        outs = [p.communicate()[0] for p in ps]
        rcs = [p.returncode for p in ps]
        ends = [float(o.split()[-1]) for o in outs if o.split()]
        wall = (max(ends) - t_go) if len(ends) == procs else float("nan")
    med = statistics.median(ts)
    return {"value": round(D / med / 1e6, 2), "unit": "MB/s", "cores": 1, "ok": bool(ok),
            "sample": (f"linApproach(jumpbits={jumpbits}) on the {mib} MiB kjv-tiled stream ({D} B decoded; "
                       f"the largest the HUFF header's int32 bit count holds), median of {reps}"),
            "processes": {"n": procs, "ok": all(r == 0 for r in rcs),
                          "value": round(procs * 2 * D / wall / 1e6, 1), "unit": "MB/s",
                          "wall_s": round(wall, 2),
                          "sample": (f"{procs} processes started together (after each loaded the "
                                     f"file), each decoding the whole stream twice; wall time to the "
                                     f"last one's end; host cores: {os.cpu_count()} visible")}}


def phase_split(device: int, tree, flags: int, data, bits: int, out, n: int = 3) -> dict:
    """Count / scan / emission device times of the TWO-PASS form, from a
    separate decoder with HH_FLAG_PHASE_TIMING (events between its kernels,
    ~6 us of idle GPU each: never in the timed decodes), after the timed
    region.  (The single pass is one kernel: no split.)"""
    import torch
    import huffmandecoderongpus_amd as H
    d = H.Decoder(device, flags=flags | H.FLAG_PHASE_TIMING)
    try:
        d.set_tree(tree)
        d.decode_device(data, bits, out)
        st = []
        for _ in range(n):
            d.decode_device(data, bits, out)
            st.append(d.stats())
        torch.cuda.synchronize()
    finally:
        d.close()
    return {k: round(statistics.mean(s[f"ms_{k}"] for s in st), 4) for k in ("sync", "scan", "emit", "total")}


def device_workload(name: str, dec, data, bits: int, out, n_want: int, verify, steps: int,
                    warmup: int, tree=None, flags: int = 0, device: int = 0) -> dict:
    """One more single-GPU workload, device-resident like the headline one:
    correctness first, then `steps` timed decodes as a stream of
    asynchronous decodes (kernel time from the decoder's HIP events, wall
    time around the loop, every decode's length checked)."""
    import torch
    n = dec.decode_device(data, bits, out)
    torch.cuda.synchronize()
    ok = n == n_want and verify(out)
    for _ in range(warmup):
        dec.decode_device(data, bits, out)
    torch.cuda.synchronize()
    st, lens = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        lens.append(dec.decode_device_async(data, bits, out))   # (as the headline loop)
        if len(lens) > 1:
            st.append(dec.stats())
    dec.wait()
    st.append(dec.stats())
    torch.cuda.synchronize()
    ms_step = (time.perf_counter() - t0) / steps * 1e3
    ok = ok and all(int(x.value) == n_want for x in lens)
    ms_dev = statistics.mean(s["ms_total"] for s in st)
    C = (bits + 7) // 8
    ach = (C + n_want) / (ms_dev * 1e-3) / 1e9
    ph = phase_split(device, tree, flags, data, bits, out) if tree is not None else None
    return {"workload": name, "ok": bool(ok), "value": round(n_want / (ms_step * 1e-3) / 1e6, 1),
            "unit": "MB/s", "ms_per_step": round(ms_step, 4), "ms_kernel": round(ms_dev, 4),
            "ms_front": ph["sync"] if ph else None, "ms_emit": ph["emit"] if ph else None,
            "compressed_bytes": C, "decoded_bytes": n_want,
            "roofline_frac": round(ach / HBM_PEAK_GBS, 4),
            "fast_path": all(s["exact_fallback"] == 0 for s in st),
            "fixed_length_path": all(s["fixed_length"] == 1 for s in st),
            "state_machine_path": all(s["state_machine"] in (1, 2) for s in st),
            "single_pass": all(s["state_machine"] == 2 for s in st)}


def gpu_local_cpus(device: int = 0):
    """The host CPUs on the GPU's NUMA node that this process may run on
    (None if unknown): hipDeviceGetPCIBusId -> /sys/bus/pci/devices/<id>/
    local_cpulist, intersected with the process's affinity."""
    import ctypes
    try:
        import torch  # noqa: F401  (its HIP runtime is the one loaded)
        hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return None
        bus = buf.value.decode().lower()
        with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
            spec = f.read().strip()
        cpus = set()
        for part in spec.split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        return cpus or None
    except (OSError, ValueError, AttributeError):
        return None


def evaluate_scope(H, hf, payload, bits: int, n_want: int, reps: int, check=None) -> dict:
    """The reference's evaluate() scope: the whole decoder call is timed
    (decodeUtil.c:41-43, 57-59) with the output buffer allocated and cleared
    beforehand (decodeUtil.c:37-38, 55); host payload in, host symbols out,
    through hh_decode_host (chunked uploads, per-chunk decodes and downloads
    overlapped).  Both the median and the reference's min over repeats are
    reported.  The decoder keeps the caller's two buffers page-locked across
    the calls (HH_FLAG_KEEP_HOST_PINNED: registered by the first call, as
    evaluate() reuses the same buffers for its 25 repeats) instead of
    registering ~3 GB in every call."""
    import numpy as np
    # the caller's buffers on the GPU's NUMA node (first touch by a thread
    # running there): DMA from the other socket's memory ran at about half
    # the rate (68 against 39 ms per 1 GiB call in round 4's runs)
    local = gpu_local_cpus(0)
    keep_aff = os.sched_getaffinity(0)
    if local:
        os.sched_setaffinity(0, local)
    payload = np.array(payload, np.uint8, copy=True)
    dec = H.Decoder(0, flags=H.FLAG_KEEP_HOST_PINNED)
    try:
        dec.set_tree(hf.tree())
        buf = np.zeros(n_want + 16, np.uint8)
        buf[:] = 0
        out = dec.decode_host(payload, bits, n_want + 16, out=buf)   # first call: allocations
        ok = len(out) == n_want and (check is None or check(out))
        ts = []
        for _ in range(reps):
            buf[:] = 0
            t0 = time.perf_counter()
            out = dec.decode_host(payload, bits, n_want + 16, out=buf)
            ts.append(time.perf_counter() - t0)
        del out, buf
        ms = statistics.median(ts) * 1e3
        return {"ok": bool(ok), "ms": round(ms, 3), "ms_min": round(min(ts) * 1e3, 3),
                "ms_max": round(max(ts) * 1e3, 3),
                "MBps": round(n_want / (ms * 1e-3) / 1e6, 1), "decoded_bytes": n_want, "reps": reps,
                "host_buffers": "page-locked once, kept across calls (HH_FLAG_KEEP_HOST_PINNED)",
                "numa_local_cpus": len(local) if local else None}
    finally:
        dec.close()
        os.sched_setaffinity(0, keep_aff)


def encode_rate(H, hf, text, n: int, dev, reps: int = 5) -> dict:
    """The device encoder (hh_encode_device) on the headline's symbols (the
    kjv text tiled to n bytes, resident in HBM) with kjv.txt.huff's codes:
    wall time per call (it synchronises), the stream checked against the
    decoder's input bits.  HBM-bound: 1 B read per symbol, its bits
    written, plus the output's zeroing."""
    import numpy as np
    import torch
    tree = hf.tree()
    t = torch.from_numpy(np.ascontiguousarray(text)).to(dev)
    syms = t.repeat(n // t.numel() + 1)[:n]
    del t
    out = torch.empty((n * 24 + 31) // 32 * 4 + 64, dtype=torch.uint8, device=dev)
    bits = H.encode_device(tree, syms, out)
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        H.encode_device(tree, syms, out)
        ts.append(time.perf_counter() - t0)
    ms = statistics.median(ts) * 1e3
    dec = H.Decoder(dev.index or 0)
    try:
        dec.set_tree(tree)
        back = torch.empty(n + 4096, dtype=torch.uint8, device=dev)
        ok = dec.decode_device(out, bits, back) == n and bool(torch.equal(back[:n], syms))
        del back
    finally:
        dec.close()
    del out, syms
    torch.cuda.empty_cache()
    return {"ok": ok, "symbols": n, "bits": bits, "ms": round(ms, 3),
            "symbols_MBps": round(n / (ms * 1e-3) / 1e6, 1),
            "hbm_GBps": round((n + 2 * (bits + 7) // 8) / (ms * 1e-3) / 1e9, 1)}


def copy_rate(dev, nbytes: int, reps: int = 5) -> dict:
    """The HBM rate a plain stream reaches on this GPU, for `frac_vs_copy`
    (BASELINE.md 3): hh_copy_device -- one 16-B load and store per lane,
    n / 256 workgroups of 256 (the fastest shape tools/ubench/ub_copy.hip
    found) -- copying `nbytes` (read + write = 2 x nbytes moved), plain and
    nontemporal, median of `reps` each; the faster of the two is the
    reference."""
    import torch
    import huffmandecoderongpus_amd as H
    nbytes = nbytes // 16 * 16
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    torch.cuda.synchronize()
    res = {}
    for nt in (False, True):
        H.copy_device(a, b, nt)
        ts = [H.copy_device(a, b, nt) for _ in range(reps)]
        res["nt" if nt else "plain"] = round(2 * nbytes / (statistics.median(ts) * 1e-3) / 1e9, 1)
    del a, b
    torch.cuda.empty_cache()
    best = max(res.values())
    return {"GBps": best, "by_policy": res, "bytes_moved": 2 * nbytes,
            "kernel": "hh_copy_device (one 16-B element per lane, n / 256 workgroups of 256, no grid-stride loop)"}


def load_pmc(path: str, workload: str):
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_decode")
    except (OSError, ValueError):
        pass
    return None


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a) -> int:
    """`bench.py --gpus N` started as a plain process (WORLD_SIZE unset):
    start N ranks under torch.distributed.run as a CHILD process -- before
    anything here touches the GPU -- and return its exit code.  Fails loudly
    when the node has fewer than N GPUs (torch.cuda.device_count() does not
    initialise the GPU on this image)."""
    import subprocess
    import torch
    have = torch.cuda.device_count()
    if have < a.gpus and not a.one_device:
        raise SystemExit(f"bench.py --gpus {a.gpus}: only {have} GPU(s) visible on this node")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def main():
    a = _args()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:
        if a.gpus > 1:
            sys.exit(launch_ranks(a))
        world = 1
    if world != a.gpus:
        raise SystemExit(f"bench.py --gpus {a.gpus} but WORLD_SIZE={world}")
    import torch
    import torch.distributed as dist
    import huffmandecoderongpus_amd as H
    from huffmandecoderongpus_amd import synth

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.one_device:
        if a.backend != "gloo":
            raise SystemExit("bench.py --one-device needs --backend gloo (RCCL refuses two ranks on one GPU)")
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(a.backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    hf, text = synth.load_source(a.files, "kjv.txt", device=local)
    target = a.size_mib << 20
    if world > 1:
        from huffmandecoderongpus_amd import shard as SH
        job = SH.ShardJob(hf, text, target, rank, world, local)
        run_step = job.check_step
        C_bytes, D_bytes = job.compressed_bytes, job.decoded_bytes
        dec = job.dec
    else:
        syn = synth.tiled_stream(hf, text, target, device=dev)
        dec = H.Decoder(local)
        dec.set_tree(syn.tree)
        out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev)
        C_bytes, D_bytes = syn.compressed_bytes, syn.decoded_bytes

        def run_step():
            return dec.decode_device(syn.data, syn.bits, out, stream)

        def run_step_async():
            # enqueues this decode and checks the previous one (its length,
            # status and device times) while this one runs
            return dec.decode_device_async(syn.data, syn.bits, out, stream)

    # correctness of the measured configuration, outside the timed region
    n = run_step()
    torch.cuda.synchronize()
    if world > 1:
        ok = job.verify()
        D_bytes = job.decoded_bytes       # known once the shard has been decoded
    else:
        ok = n == syn.decoded_bytes and synth.verify_tiled(out, syn)
    if not ok:
        raise SystemExit(f"rank {rank}: decoded output does not match the tiled text")

    if world > 1:
        job.pipelined_steps(a.warmup)       # (the timed form: decode, exchange, any redo)
    else:
        for _ in range(a.warmup):
            run_step()
    torch.cuda.synchronize()
    # (collectives over host tensors with gloo)
    red_dev = torch.device("cpu") if world > 1 and a.backend == "gloo" else dev
    sync_ms = None
    if world == 1:
        # the synchronous call (hh_decode_device: returns once the length is
        # known) timed on its own, for the per-call latency
        ts = []
        for _ in range(max(3, a.steps // 2)):
            t1 = time.perf_counter()
            run_step()
            ts.append(time.perf_counter() - t1)
        sync_ms = statistics.median(ts) * 1e3
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dev_ms, lens = [], []
    t0 = time.perf_counter()
    if world == 1:
        # a stream of decodes: each enqueued while the previous one runs and
        # is checked (hh_decode_device_async), the last checked by the wait
        for _ in range(a.steps):
            lens.append(run_step_async())
            if len(lens) > 1:
                dev_ms.append(dec.stats())      # (the decode checked by this call)
        dec.wait()
        dev_ms.append(dec.stats())
    else:
        # a full step per rank: its shard's decode (prologue + owned tiles,
        # entered in the guessed state), the entry exchange (5 integers,
        # all-gather: it proves every entry and gives the output bases) and
        # the redo of a wrong entry -- nothing carried over from the checked
        # step; every step's rows must equal the checked step's.  Pipelined:
        # step k's exchange and redo run while step k+1's decode is in flight
        # (shard.pipelined)
        steps_ok = job.pipelined_steps(a.steps)
        dev_ms.append(dec.stats())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world == 1 and any(int(n.value) != syn.decoded_bytes for n in lens):
        raise SystemExit("a timed decode returned the wrong length")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_step = elapsed / a.steps * 1e3
    ms_dev = statistics.mean(s["ms_total"] for s in dev_ms)
    # the split by kernel from a separate phase-timed decoder (world 1)
    phases = (phase_split(local, syn.tree, 0, syn.data, syn.bits, out) if world == 1
              else {"sync": None, "scan": None, "emit": None})
    fast = all(s["exact_fallback"] == 0 for s in dev_ms)
    kernels = ("k_one" if all(s["state_machine"] == 2 for s in dev_ms)
               else "k_cntm+k_fscan1+k_emf" if all(s["state_machine"] for s in dev_ms)
               else "k_front+k_walk+k_table+k_scan1+k_scan2+k_emit")
    extra = {}
    if world > 1:
        # the decode alone (the figure for the decode-time scaling target):
        # each rank's shard decodes queued asynchronously, entered in the
        # settled entry -- no exchange inside; the exchange over the last
        # one's results after the region must reproduce the checked rows
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(a.steps):
            job.decode_step()
        job.wait()
        torch.cuda.synchronize()
        dist.barrier()
        td = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=red_dev)
        dist.all_reduce(td, op=dist.ReduceOp.MAX)
        confirmed = torch.tensor([1 if (job.confirm() and steps_ok) else 0], dtype=torch.int64, device=red_dev)
        dist.all_reduce(confirmed, op=dist.ReduceOp.MIN)
        extra = job.gather_report()
        ms_dec = float(td.item()) / a.steps * 1e3
        extra["settle"] = {"timed_step": "decode + 5-integer entry all-gather + any redo, every step; step k's "
                                         "exchange and redo overlap step k+1's decode (job.pipelined_steps)",
                           "redo_on_checked_step": job.redo_state is not None,
                           "confirmed_after_timed": bool(confirmed.item()),
                           "decode_only": {"ms_per_step": round(ms_dec, 4),
                                           "note": "shard decodes alone, entered in the settled entry, "
                                                   "queued asynchronously; the exchange after them"}}
        if not confirmed.item():
            raise SystemExit(f"rank {rank}: the entry exchange of a timed step disagrees with the checked one")
        tot = torch.tensor([C_bytes, D_bytes], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tot)
        C_all, D_all = int(tot[0].item()), int(tot[1].item())
    else:
        C_all, D_all = C_bytes, D_bytes
    workload = f"synthetic {a.size_mib} MiB/GPU kjv-tiled .huff"
    achieved = (C_bytes + D_bytes) / (ms_dev * 1e-3) / 1e9
    traffic = load_pmc(a.pmc, workload)
    res = {
        "metric": "decoded MB/s",
        "value": round(D_all / (ms_step * 1e-3) / 1e6, 1),
        "unit": "MB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic: files/kjv.txt tiled and encoded with the kjv.txt.huff "
                 "codebook (payload bit-concatenation), cut at a symbol boundary"),
        "config": {"workload": workload + (f", sharded over {world} GPUs" if world > 1 else ", 1 MI355X"),
                   "compressed_bytes": C_all, "decoded_bytes": D_all,
                   "bits_per_gpu": int(C_bytes * 8), "parallelism": f"byte-range shards x{world}"},
        "roofline": {"bound": "hbm", "kernel": kernels,
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_alg": C_bytes + D_bytes, "ms_kernel": round(ms_dev, 4),
                     "two_pass_split_ms": {"count": phases["sync"], "scan": phases["scan"],
                                           "emit": phases["emit"]}},
        "decoded_MBps_device": round(D_bytes / (ms_dev * 1e-3) / 1e6, 1),
        "ms_per_call_sync": round(sync_ms, 4) if sync_ms is not None else None,
        "fast_path": fast,
        "state_machine_path": all(s["state_machine"] in (1, 2) for s in dev_ms),
        "single_pass": all(s["state_machine"] == 2 for s in dev_ms),
    }
    res.update(extra)
    if world == 1:
        # the same box's streaming rate over the same bytes (after the timed region)
        cp = copy_rate(dev, (C_bytes + D_bytes) // 2)
        res["roofline"]["copy_GBps"] = cp["GBps"]
        res["roofline"]["copy"] = cp
        res["roofline"]["frac_vs_copy"] = round(achieved / cp["GBps"], 4)
    if world == 1 and not a.no_extra:
        # SURVEY 8d's other single-GPU configs and the evaluate() scope
        # (after the headline measurement, outside its timed region)
        import numpy as np
        del out
        torch.cuda.empty_cache()
        # evaluate() scope: kjv.txt.huff itself, and the headline 1 GiB stream
        # from host memory -- first, while the host has its memory to itself
        # (run after the workloads below, the 1 GiB call took 68 ms, 39 here)
        ev = {"kjv.txt": evaluate_scope(H, hf, hf.payload, hf.bits, hf.uncompressedsize, 20,
                                        lambda o: np.array_equal(o, text))}
        host_pay = syn.data[: syn.compressed_bytes].cpu().numpy()
        ev[f"{a.size_mib} MiB kjv-tiled"] = evaluate_scope(
            H, hf, host_pay, syn.bits, syn.decoded_bytes, 5,
            lambda o: synth.verify_tiled(torch.from_numpy(o).to(dev), syn))
        del host_pay
        res["evaluate"] = ev
        ks = max(3, min(a.steps, 10))
        more = []
        hfe, texte = synth.load_source(a.files, "E.coli", device=local)
        syn_e = synth.tiled_stream(hfe, texte, target, device=dev)
        dec_e = H.Decoder(local)
        dec_e.set_tree(syn_e.tree)
        out_e = torch.empty(syn_e.decoded_bytes + 4096, dtype=torch.uint8, device=dev)
        more.append(device_workload(f"synthetic {a.size_mib} MiB E.coli-tiled .huff", dec_e,
                                    syn_e.data, syn_e.bits, out_e, syn_e.decoded_bytes,
                                    lambda o: synth.verify_tiled(o, syn_e), ks, 2, syn_e.tree, 0, local))
        dec_e.close()
        # the same stream through the general pipeline (heads, exit merges,
        # walks, tables, scans, emission): config 5's merge-density stress
        dec_g = H.Decoder(local, flags=H.FLAG_NO_FIXED)
        dec_g.set_tree(syn_e.tree)
        more.append(device_workload(f"synthetic {a.size_mib} MiB E.coli-tiled .huff, general pipeline "
                                    f"(HH_FLAG_NO_FIXED)", dec_g, syn_e.data, syn_e.bits, out_e,
                                    syn_e.decoded_bytes, lambda o: synth.verify_tiled(o, syn_e), ks, 2,
                                    syn_e.tree, H.FLAG_NO_FIXED, local))
        dec_g.close()
        del out_e, syn_e
        torch.cuda.empty_cache()
        iid = synth.iid_stream(hf, text, target, device=dev)
        out_i = torch.empty(iid.decoded_bytes + 4096, dtype=torch.uint8, device=dev)
        more.append(device_workload(f"synthetic {a.size_mib} MiB i.i.d. kjv-unigram .huff "
                                    f"(splitmix64 seed {synth.IID_SEED:#x})", dec, iid.data,
                                    iid.bits, out_i, iid.decoded_bytes,
                                    lambda o: bool(torch.equal(o[:iid.decoded_bytes], iid.syms)),
                                    ks, 2, iid.tree, 0, local))
        del out_i, iid
        torch.cuda.empty_cache()
        # a byte alphabet: Huffman code over all 256 byte values (255 states,
        # the state machine's 7-bit count steps over 224-bit regions)
        byt = synth.byte_stream(target, device=dev)
        dec_b = H.Decoder(local)
        dec_b.set_tree(byt.tree)
        out_b = torch.empty(byt.decoded_bytes + 4096, dtype=torch.uint8, device=dev)
        more.append(device_workload(f"synthetic {a.size_mib} MiB byte-alphabet .huff (256-symbol Huffman "
                                    f"code, Zipf s={synth.ZIPF_S} byte frequencies, splitmix64 seed "
                                    f"{synth.BYTE_SEED:#x})", dec_b, byt.data, byt.bits, out_b,
                                    byt.decoded_bytes,
                                    lambda o: bool(torch.equal(o[:byt.decoded_bytes], byt.syms)), ks, 2,
                                    byt.tree, 0, local))
        dec_b.close()
        del out_b, byt
        torch.cuda.empty_cache()
        res["workloads"] = more
        res["encode"] = encode_rate(H, hf, text, syn.decoded_bytes, dev)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(a.files, a.cpu_seconds)
        from oracle import oracle as O
        if O.ref_available():
            res["cpu_baseline"]["tiled"] = cpu_baseline_tiled(
                H, hf, text, 128, res["cpu_baseline"]["jumpbits"], 3, min(16, os.cpu_count() or 1))
        if "workloads" in res:
            # beside the E.coli workload: the reference's best jumpbits differs there
            res["workloads"][0]["cpu_baseline"] = cpu_baseline(a.files, a.cpu_seconds, "E.coli.huff")
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
