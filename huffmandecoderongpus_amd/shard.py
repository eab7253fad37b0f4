"""Multi-GPU decode: the stream cut into byte ranges of whole tiles, one
process (rank) per GPU (the reference has no multi-device
path, its single-device host orchestration is openclapproach.c:236-1047).

A rank owns tiles [t0, t1) of the global tile grid (hh_decoder_tile_bits
bits each).  Ranges are independent except for one thing: the state in which
the decode chain ENTERS the range (region, offset, count correction), which
is the state leaving the previous range.  Each rank finds it locally: its
buffer starts PROBE tiles before t0, and those tiles are decoded as a
prologue (hh_range.prologue) -- their transfer tables give the entry state
exactly whenever one of them is CONST (leaving state independent of how it
was entered), which natural codes almost always are.  The ranks then
exchange (entry, leave, exactness, symbol count) -- 5 integers each, one
all-gather -- which (a) proves every entry against the predecessor's leave
state and lets a rank entered wrongly decode again with the right one (in
at most world-1 more rounds; never needed when the prologue was exact), and
(b) gives every rank its output base (exclusive sum of symbol counts).  The
data path has no collective; assembling the global output is one all-gather
of the decoded segments, timed separately (bench.py gather_report).

The settle protocol is pure Python over a `gather` callable so that it is
tested with gloo on CPU (tests/test_shard.py) against the kernel's host
emulation; the device path is ShardJob.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np

PROBE_TILES = 2          # predecessor tiles decoded as a prologue


@dataclass
class Segment:
    """Rank-local view of a shard.  Bit positions are global."""
    rank: int
    world: int
    t0: int              # first owned tile
    t1: int              # one past the last owned tile
    tile_bits: int
    total_bits: int      # global stream length
    prologue: int        # predecessor tiles at the start of the local buffer

    @property
    def buf_bit(self) -> int:          # global bit of the local buffer's start
        return (self.t0 - self.prologue) * self.tile_bits

    @property
    def ntiles(self) -> int:           # tiles decoded (prologue + owned)
        return self.prologue + self.t1 - self.t0

    @property
    def bits_avail(self) -> int:       # owned tiles + one tile of halo, or to the end
        return min(self.total_bits - self.buf_bit, (self.ntiles + 1) * self.tile_bits)

    @property
    def owned_bits(self) -> int:
        return min(self.total_bits, self.t1 * self.tile_bits) - self.t0 * self.tile_bits


def plan(total_bits: int, tile_bits: int, world: int, rank: int,
         probe: int = PROBE_TILES) -> Segment:
    """Near-equal contiguous tile ranges; rank r > 0 also holds `probe`
    tiles of its predecessor."""
    nt = (total_bits + tile_bits - 1) // tile_bits
    t0, t1 = rank * nt // world, (rank + 1) * nt // world
    pro = min(probe, t0) if rank > 0 else 0
    return Segment(rank, world, t0, t1, tile_bits, total_bits, pro)


def settle(first: dict, redo, gather, rank: int, world: int) -> tuple[dict, list]:
    """Make every rank's entry state exact.

    first   this rank's result: in_state, leave_state, entry_exact,
            const_seen, out_len
    redo    redo(in_state) -> result: decode the owned tiles only, entered
            in in_state
    gather  gather(list of 5 ints) -> list of world such lists (all ranks)

    Returns (this rank's final result, all ranks' final rows).  A rank's
    entry is right when it is rank 0, or its prologue was exact, or it equals
    the predecessor's leave state and that leave state is valid (the
    predecessor's entry is right, or its own tables make its leave state
    independent of the entry)."""
    res = dict(first)
    for _ in range(world + 1):
        rows = gather([res["in_state"], res["leave_state"], int(res["entry_exact"]),
                       int(res["const_seen"]), res["out_len"]])
        right = [False] * world
        fix = {}
        for r in range(world):
            ins, _, exact, _, _ = rows[r]
            if r == 0 or exact:
                right[r] = True
                continue
            p = rows[r - 1]
            prev_valid = right[r - 1] or bool(p[3])
            if not prev_valid:
                continue
            if ins == p[1]:
                right[r] = True
            else:
                fix[r] = p[1]
        if all(right):
            return res, rows
        if rank in fix:
            res = redo(fix[rank])
            res["entry_exact"] = True        # entered in the predecessor's valid leave state
    raise RuntimeError("shard entry states did not settle")


def out_base(rows: list, rank: int) -> int:
    return int(sum(int(rows[r][4]) for r in range(rank)))


def assemble(local, n: int, rows: list, dist, world: int):
    """The global output from the ranks' segments: one all-gather of the
    segments padded to the largest (RCCL: all_gather_into_tensor on the
    GPU; gloo: host tensors), then rank r's first out_len bytes in rank
    order.  `local` is this rank's segment buffer (n bytes valid).  Returns
    (the gathered padded buffer, the padded length)."""
    import torch
    mx = max(int(r[4]) for r in rows)
    gloo = dist.get_backend() == "gloo"
    dev = torch.device("cpu") if gloo else local.device
    pad = torch.zeros(max(mx, 1), dtype=torch.uint8, device=dev)
    pad[:n] = local[:n].to(dev)
    if gloo:
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
        big = torch.cat(parts)
    else:
        big = torch.empty(pad.numel() * world, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(big, pad)
    return big, pad.numel()


def concat(big, mx: int, rows: list):
    """The stream's symbols from assemble()'s buffer."""
    import torch
    return torch.cat([big[r * mx:r * mx + int(rows[r][4])] for r in range(len(rows))])


class ShardJob:
    """One rank's shard of the synthetic workload on its GPU: the global
    stream is `world` x target_bytes of tiled kjv.txt (cut at a symbol), this
    rank decodes its tiles (bench.py --gpus N)."""

    def __init__(self, hf, text: np.ndarray, target_bytes: int, rank: int, world: int,
                 local: int, probe: int = PROBE_TILES):
        import torch
        import torch.distributed as dist
        import huffmandecoderongpus_amd as H
        from huffmandecoderongpus_amd import synth
        self.rank, self.world = rank, world
        self.dev = torch.device("cuda", local)
        self.dec = H.Decoder(local)
        self.tree = hf.tree()
        self.dec.set_tree(self.tree)
        tb = self.dec.tile_bits()
        total_bits, total_syms = synth.cut_bits(hf, text, world * target_bytes)
        self.seg = plan(total_bits, tb, world, rank, probe)
        s = self.seg
        self.syn = synth.tiled_stream(hf, text, 0, device=self.dev, bit_offset=s.buf_bit,
                                      bits=s.bits_avail)
        self.text = self.syn.text
        self.total_syms = total_syms
        minlen = int(min(v for v in synth.code_lengths(self.tree) if v > 0))
        self.cap = s.owned_bits // minlen + 4096
        self.out = torch.empty(self.cap, dtype=torch.uint8, device=self.dev)
        self.stream = torch.cuda.current_stream(self.dev)
        self.compressed_bytes = (s.owned_bits + 7) // 8
        self.decoded_bytes = 0
        self.rows = None
        self._dist = dist

    def _gather(self, vals):
        import torch
        cpu = self._dist.get_backend() == "gloo"      # gloo: host tensors
        t = torch.tensor(vals, dtype=torch.int64, device="cpu" if cpu else self.dev)
        allt = [torch.empty_like(t) for _ in range(self.world)]
        self._dist.all_gather(allt, t)
        return [[int(v) for v in a.tolist()] for a in allt]

    def _decode(self, in_state: int, prologue: int) -> dict:
        s = self.seg
        skip = (s.prologue - prologue) * s.tile_bits          # bits, multiple of 32
        # (no owned tile, fewer tiles than ranks: ntiles 0, and the range
        # decode leaves the chain in the state it entered)
        nt = s.ntiles - (s.prologue - prologue) if s.t1 > s.t0 else 0
        r = self.dec.decode_range_ptr(self.syn.data.data_ptr() + skip // 8,
                                      s.bits_avail - skip, nt, in_state, self.out.data_ptr(),
                                      self.cap, self.stream.cuda_stream, prologue=prologue)
        r["in_state"] = r["entry_state"]
        return r

    def decode_step(self) -> int:
        """One decode of this rank's shard, entry states settled (timed)."""
        s = self.seg
        first = self._decode(0, s.prologue)
        if s.prologue == 0 and s.t0 > 0:
            first["entry_exact"] = False      # no prologue: the entry is a guess
        res, rows = settle(first, lambda st: self._decode(st, 0), self._gather,
                           self.rank, self.world)
        self.rows = rows
        self.decoded_bytes = res["out_len"]
        return res["out_len"]

    def verify(self) -> bool:
        """Output == the tiled text from this rank's global symbol index."""
        import torch
        if self.rows is None:
            return False
        base = out_base(self.rows, self.rank)
        n = self.decoded_bytes
        if self.rank == self.world - 1 and base + n != self.total_syms:
            return False
        L = self.text.numel()
        step = 1 << 28
        for o in range(0, n, step):
            m = min(step, n - o)
            idx = (torch.arange(m, device=self.dev, dtype=torch.int64) + (base + o)) % L
            if not torch.equal(self.out[o:o + m], self.text[idx]):
                return False
        return True

    def gather_report(self) -> dict:
        """All-gather of the decoded segments (assemble()), timed outside
        the decode steps: the assembly cost, reported separately.  Rank 0
        then checks every rank's part of the assembled stream against the
        tiled text from that rank's base."""
        import torch
        n = self.decoded_bytes
        self._dist.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        big, mx = assemble(self.out, n, self.rows, self._dist, self.world)
        if big.is_cuda:
            torch.cuda.synchronize(self.dev)
        t = time.perf_counter() - t0
        tt = torch.tensor([t], dtype=torch.float64)
        if self._dist.get_backend() != "gloo":
            tt = tt.to(self.dev)
        self._dist.all_reduce(tt, op=self._dist.ReduceOp.MAX)
        t = float(tt.item())
        ok = True
        if self.rank == 0:
            L = self.text.numel()
            text = self.text.to(big.device)
            step = 1 << 28
            for r in range(self.world):
                b, k = out_base(self.rows, r), int(self.rows[r][4])
                for o in range(0, k, step):
                    m = min(step, k - o)
                    idx = (torch.arange(m, device=big.device, dtype=torch.int64) + (b + o)) % L
                    ok = ok and torch.equal(big[r * mx + o:r * mx + o + m], text[idx])
            ok = ok and out_base(self.rows, self.world) == self.total_syms
        del big
        torch.cuda.empty_cache()
        return {"allgather": {"ms": round(t * 1e3, 3), "bytes_per_rank": mx * self.world,
                              "GBps_in_per_rank": round(mx * (self.world - 1) / max(t, 1e-9) / 1e9, 1),
                              "seams_ok": bool(ok)}}
