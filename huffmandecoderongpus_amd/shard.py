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
(b) gives every rank its output base (exclusive sum of symbol counts).

Every step bench.py times is a full step (full_step): the decode, the
exchange and any redo, nothing carried over from an earlier step; its rows
must reproduce those of the CHECKED step before the timed region
(check_step).  bench.py also times the decodes alone (decode_step: the
prologue decode, plus the redo from the settled entry when the checked step
needed one, queued asynchronously with no collective; the exchange over
the last one's results afterwards, confirm, must reproduce the checked
rows) and reports them apart, as the decode-time figure.  Assembling the
global output is one all-gather of the decoded segments, timed separately
(bench.py gather_report).

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


def check_settle(first: dict, redo, gather, rank: int, world: int):
    """The checked step's exchange: settle(), plus the state this rank was
    redone from (None: its first entry was right).  Returns (result, rows,
    redo_state)."""
    called = []

    def rec(st):
        called.append(st)
        return redo(st)
    res, rows = settle(first, rec, gather, rank, world)
    return res, rows, (called[-1] if called else None)


def confirm(first: dict, redone: dict, gather, rank: int, world: int, rows_ref: list) -> bool:
    """After the timed steps: the settle exchange over the last timed step's
    results -- `first` its prologue decode, `redone` {state: result} of the
    redo it queued -- must end with the checked step's rows and ask for no
    decode the timed step did not do.  Collective (every rank calls it)."""
    missing = []

    def redo(st):
        if st in redone:
            return redone[st]
        missing.append(st)
        return {"in_state": st, "leave_state": -1, "entry_exact": True, "const_seen": False, "out_len": -1}
    try:
        _, rows = settle(first, redo, gather, rank, world)
    except RuntimeError:
        return False
    return not missing and [list(map(int, r)) for r in rows] == [list(map(int, r)) for r in rows_ref]


def pipelined(steps: int, launch, settle_one, wait) -> list:
    """Full steps, pipelined: step k's decode is enqueued (launch(k) returns
    its handle, whose results are valid once the next launch has returned or
    wait() has), then step k-1 is settled -- its entry exchange and any redo,
    settle_one(handle) -> its rows -- while step k's decode runs.  Every step
    gets its own decode, exchange and redo; only their overlap changes.
    Returns every step's rows, in step order.  Collective when settle_one is."""
    got, prev = [], None
    for k in range(steps):
        h = launch(k)
        if prev is not None:
            got.append(settle_one(prev))
        prev = h
    wait()
    if prev is not None:
        got.append(settle_one(prev))
    return got


def _rows_eq(a: list, b: list) -> bool:
    return [list(map(int, r)) for r in a] == [list(map(int, r)) for r in b]


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
                 local: int, probe: int = PROBE_TILES, wrong_entry: bool = False):
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
        self.out2 = None                # (pipelined_steps: the other step's output)
        # the shard decodes on a stream of their own: a collective over
        # device tensors (RCCL) waits for the current stream's work, and the
        # pipelined steps' exchange must not wait for the next decode
        self.stream = torch.cuda.Stream(self.dev)
        self.compressed_bytes = (s.owned_bits + 7) // 8
        self.decoded_bytes = 0
        self.rows = None
        self.redo_state = None
        self.last_rows = self.last_redo = None
        self._last = None
        self._dist = dist
        # tests: a rank without a prologue enters in a state known to be
        # wrong (its true entry found by a prologue decode here), so that the
        # exchange must catch it and the timed steps include the redo
        self.guess = 0
        if wrong_entry and s.prologue == 0 and s.t0 > 0 and s.t1 > s.t0:
            k = min(PROBE_TILES, s.t0)
            pro = synth.tiled_stream(hf, text, 0, device=self.dev, bit_offset=(s.t0 - k) * tb,
                                     bits=min(total_bits - (s.t0 - k) * tb, (k + 2) * tb))
            r = self.dec.decode_range_ptr(pro.data.data_ptr(), pro.bits, k + 1, 0, self.out.data_ptr(),
                                          self.cap, self.stream.cuda_stream, prologue=k)
            del pro
            self.guess = 1 if r["entry_state"] == 0 else 0

    def _gather(self, vals):
        import torch
        cpu = self._dist.get_backend() == "gloo"      # gloo: host tensors
        t = torch.tensor(vals, dtype=torch.int64, device="cpu" if cpu else self.dev)
        allt = [torch.empty_like(t) for _ in range(self.world)]
        self._dist.all_gather(allt, t)
        return [[int(v) for v in a.tolist()] for a in allt]

    def _args(self, prologue: int):
        s = self.seg
        skip = (s.prologue - prologue) * s.tile_bits          # bits, multiple of 32
        # (no owned tile, fewer tiles than ranks: ntiles 0, and the range
        # decode leaves the chain in the state it entered)
        nt = s.ntiles - (s.prologue - prologue) if s.t1 > s.t0 else 0
        return self.syn.data.data_ptr() + skip // 8, s.bits_avail - skip, nt

    def _decode(self, in_state: int, prologue: int, out=None) -> dict:
        ptr, bits, nt = self._args(prologue)
        out = self.out if out is None else out
        r = self.dec.decode_range_ptr(ptr, bits, nt, in_state, out.data_ptr(), self.cap,
                                      self.stream.cuda_stream, prologue=prologue)
        r["in_state"] = r["entry_state"]
        return r

    def _launch(self, in_state: int, prologue: int, out=None):
        ptr, bits, nt = self._args(prologue)
        out = self.out if out is None else out
        return self.dec.decode_range_async_ptr(ptr, bits, nt, in_state, out.data_ptr(), self.cap,
                                               self.stream.cuda_stream, prologue=prologue)

    def _first(self, r: dict) -> dict:
        s = self.seg
        if s.prologue == 0 and s.t0 > 0:
            r["entry_exact"] = False          # no prologue: the entry is a guess
        return r

    def full_step(self) -> int:
        """One complete decode of this rank's shard: the decode entered in
        the guessed state (prologue + owned tiles), the entry-state exchange
        (settle: a 5-integer all-gather that proves every entry and gives the
        output bases), the redo of a wrong entry.  Nothing is carried over
        from an earlier step.  Collective (every rank calls it)."""
        s = self.seg
        first = self._first(self._decode(self.guess, s.prologue))
        res, rows, redo = check_settle(first, lambda st: self._decode(st, 0), self._gather, self.rank, self.world)
        self.last_rows, self.last_redo = rows, redo
        return res["out_len"]

    def check_step(self) -> int:
        """The checked decode of this rank's shard (before the timed region):
        a full step whose rows every later step must reproduce."""
        n = self.full_step()
        self.rows, self.redo_state = self.last_rows, self.last_redo
        self.decoded_bytes = n
        return n

    def pipelined_steps(self, steps: int) -> bool:
        """`steps` full steps of this rank's shard (bench.py's timed steps for
        N > 1), pipelined (shard.pipelined): step k's decode, entered in the
        guessed state, is queued on the shard's stream; step k-1's exchange
        (settle: the 5-integer all-gather) and any redo run while it is in
        flight.  Nothing is carried over between steps: each step's redo
        state comes from its own exchange.  The steps alternate between two
        output buffers (a redo never writes over the next step's output);
        the last one's is self.out.  True when every step's rows equal the
        checked step's.  Collective (every rank calls it)."""
        import torch
        if steps <= 0:
            return True
        if self.out2 is None:
            self.out2 = torch.empty_like(self.out)

        def buf(k):
            return self.out if (steps - 1 - k) % 2 == 0 else self.out2

        def launch(k):
            b = buf(k)
            return self._launch(self.guess, self.seg.prologue, b), b

        def settle_one(h):
            r, b = h
            first = r.as_dict()
            first["in_state"] = first["entry_state"]
            _, rows, redo = check_settle(self._first(first), lambda st: self._decode(st, 0, b), self._gather,
                                         self.rank, self.world)
            self.last_redo = redo
            return rows
        got = pipelined(steps, launch, settle_one, self.dec.wait)
        self.last_rows = got[-1]
        return self.rows is not None and all(_rows_eq(r, self.rows) for r in got)

    def decode_step(self) -> None:
        """One timed decode of this rank's shard: the prologue decode and, when
        the checked step's exchange found this rank's entry wrong, the redo
        from the settled entry -- queued asynchronously (the decoder checks
        the previous one meanwhile); no collective, no host wait."""
        first = self._launch(self.guess, self.seg.prologue)
        redo = self._launch(self.redo_state, 0) if self.redo_state is not None else None
        self._last = (first, redo)

    def wait(self) -> None:
        self.dec.wait()

    def confirm(self) -> bool:
        """After the timed region: the exchange over the last timed step's
        results must reproduce the checked step's rows (shard.confirm)."""
        self.dec.wait()
        first = self._last[0].as_dict()
        first["in_state"] = first["entry_state"]
        redone = {}
        if self._last[1] is not None:
            r = self._last[1].as_dict()
            r["in_state"] = r["entry_state"]
            redone[self.redo_state] = r
        return confirm(self._first(first), redone, self._gather, self.rank, self.world, self.rows)

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
