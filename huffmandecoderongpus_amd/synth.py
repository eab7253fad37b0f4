"""Synthetic workloads for the benchmark and the scale tests.

The BASELINE.json workload is "synthetic 1 GiB English-text .huff
(kjv-derived codebook)": kjv.txt tiled, encoded with the tree
of files/kjv.txt.huff.  A prefix code has no state, so the encoding of N
concatenated copies of a text is the bit-concatenation of N copies of that
text's encoding; the payload is therefore built by OR-ing bit-shifted copies
of kjv.txt.huff's payload on the GPU (no CPU encoder pass over 1.9 GB), then
cut at the last whole symbol that fits the target size.

The decoded text of kjv.txt.huff itself comes from the HIP decoder (this is
product code: the oracle is not used here) and is checked against the
sha256 recorded in BASELINE.md.
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass

import numpy as np

KJV_SHA256 = "e4e21579f6360b35e66dc97b67cd732a3f759623e41e4e077bec039eeb79fd0a"


def code_lengths(tree) -> np.ndarray:
    """Code length of every symbol byte (0 = absent), from the tree."""
    L = np.zeros(256, np.int64)
    stack = [(0, 0)]
    while stack:
        v, d = stack.pop()
        if tree.izero[v] == -1:
            if L[tree.sym[v]] == 0:
                L[tree.sym[v]] = d
        else:
            stack.append((int(tree.izero[v]), d + 1))
            stack.append((int(tree.ione[v]), d + 1))
    return L


@dataclass
class Synthetic:
    tree: object            # huffmandecoderongpus_amd.Tree
    data: object            # torch uint8 cuda tensor: payload + pad
    bits: int
    text: object            # torch uint8 cuda tensor: one copy of the source text
    copies: int             # whole copies before the partial one
    tail_syms: int          # symbols of the partial copy
    bit_offset: int         # global bit offset of this shard (multi-GPU)

    @property
    def compressed_bytes(self) -> int:
        return (self.bits + 7) // 8

    @property
    def decoded_bytes(self) -> int:
        return self.copies * int(self.text.numel()) + self.tail_syms


def load_source(files_dir: str, name: str = "kjv.txt", device: int = 0, check_sha=True):
    """(HuffFile, decoded text as numpy) for a reference fixture, via the GPU."""
    import huffmandecoderongpus_amd as H
    hf = H.HuffFile.load(os.path.join(files_dir, name + ".huff"))
    dec = H.Decoder(device)
    try:
        dec.set_tree(hf.tree())
        text = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
    finally:
        dec.close()
    if check_sha and name == "kjv.txt":
        got = hashlib.sha256(text.tobytes()).hexdigest()
        if got != KJV_SHA256:
            raise RuntimeError(f"kjv.txt decode sha256 mismatch: {got}")
    return hf, text


def cut_bits(hf, text: np.ndarray, target_bytes: int) -> tuple[int, int]:
    """(bits, symbols) of the tiled stream cut at the last whole symbol that
    fits target_bytes of payload (what tiled_stream(..., bit_offset=0) makes)."""
    B0 = hf.bits
    bounds = np.concatenate([[0], np.cumsum(code_lengths(hf.tree())[text])])
    c, within = divmod(8 * target_bytes, B0)
    k = int(np.searchsorted(bounds, within, side="right")) - 1
    return c * B0 + int(bounds[k]), c * len(text) + k


def tiled_stream(hf, text: np.ndarray, target_bytes: int, device="cuda",
                 bit_offset: int = 0, halo_bytes: int = 0, bits: int | None = None) -> Synthetic:
    """Bits [bit_offset, bit_offset + 8*target_bytes) of the infinite tiling of
    hf's payload, cut at the last whole symbol (or, with `bits`, exactly that
    many bits, no cut); plus halo_bytes more payload bytes after it (for a
    shard's successor walk).  bit_offset must be a multiple of 32 and a code
    boundary is not required there."""
    import torch
    B0 = hf.bits
    P = torch.from_numpy(hf.payload.copy()).to(device)
    lens = code_lengths(hf.tree())[text]
    bounds = np.concatenate([[0], np.cumsum(lens)])          # symbol starts + end
    assert bounds[-1] == B0
    tgt_bits = 8 * target_bytes if bits is None else bits
    gen_bits = tgt_bits + 8 * halo_bytes
    nbytes = (gen_bits + 7) // 8
    out = torch.zeros(nbytes + 64 + 8, dtype=torch.uint8, device=device)
    # copies overlapping [bit_offset, bit_offset + gen_bits)
    first = bit_offset // B0
    last = (bit_offset + gen_bits) // B0
    P16 = torch.cat([P.to(torch.int32), torch.zeros(2, dtype=torch.int32, device=device)])
    for c in range(first, last + 1):
        start = c * B0 - bit_offset          # bit position of copy c in `out`
        src_bit, dst = (0, start) if start >= 0 else (-start, 0)
        sbyte, r = divmod(src_bit, 8)
        seg = P16[sbyte:]
        if r:                                # stream bytes starting at src_bit
            seg = ((seg[:-1] >> r) | (seg[1:] << (8 - r))) & 0xff
        db, sh = divmod(dst, 8)
        n = min(seg.numel(), out.numel() - db - 1)
        if n <= 0:
            continue
        v = seg[:n] << sh
        out[db:db + n] |= (v & 0xff).to(torch.uint8)
        out[db + 1:db + n + 1] |= (v >> 8).to(torch.uint8)
    # cut the shard at the last symbol boundary <= tgt_bits
    end_global = bit_offset + tgt_bits
    cidx = end_global // B0
    within = end_global - cidx * B0
    k = int(np.searchsorted(bounds, within, side="right")) - 1   # boundaries <= within
    cut_global = cidx * B0 + int(bounds[k])
    if bits is None:
        bits = cut_global - bit_offset
    # symbols in the shard (only meaningful for bit_offset == 0)
    copies, tail = int(cidx), int(k)
    if halo_bytes == 0:
        # zero everything past the cut so the pad bytes are clean
        nb = (bits + 7) // 8
        if bits % 8:
            out[nb - 1] &= (1 << (bits % 8)) - 1
        out[nb:] = 0
    T = torch.from_numpy(text.copy()).to(device)
    return Synthetic(hf.tree(), out, bits, T, copies, tail, bit_offset)


def verify_tiled(out, syn: Synthetic) -> bool:
    """Decoded output == tiled text (checked on the GPU)."""
    import torch
    L = syn.text.numel()
    n = syn.copies * L
    if syn.copies and not torch.equal(out[:n].view(syn.copies, L),
                                      syn.text.unsqueeze(0).expand(syn.copies, L)):
        return False
    return bool(torch.equal(out[n:n + syn.tail_syms], syn.text[:syn.tail_syms]))


# ---------------------------------------------------------------------------
# i.i.d. variant: symbols drawn independently from kjv.txt's
# unigram distribution, splitmix64 with seed 0x5EED5EED.  Symbol i uses the
# generator output after i+1 increments (counter form, so every symbol is
# drawn in parallel): z = mix(seed + (i+1) * 0x9E3779B97F4A7C15), r = z >> 32,
# x = (r * T) >> 32 with T the text length, symbol = the byte b whose
# cumulative count range [cum[b-1], cum[b]) holds x.  Encoded on the GPU with
# the kjv.txt.huff codebook (codes LSB-first, the stream's bit order).
# ---------------------------------------------------------------------------
IID_SEED = 0x5EED5EED
_GOLDEN = 0x9E3779B97F4A7C15
_M1 = 0xBF58476D1CE4E5B9
_M2 = 0x94D049BB133111EB


def _s64(v: int) -> int:
    """uint64 constant as the int64 torch arithmetic wraps in."""
    return v - (1 << 64) if v >= 1 << 63 else v


def _srl(z, k: int):
    """Logical right shift of int64 tensors holding uint64 bit patterns."""
    return (z >> k) & ((1 << (64 - k)) - 1)


def splitmix64(idx, seed: int = IID_SEED):
    """splitmix64 outputs for counters idx (int64 tensor, 0-based) as int64
    bit patterns (torch) -- the numpy twin is splitmix64_np."""
    z = idx.add(1).mul(_s64(_GOLDEN)).add(_s64(seed))
    z = (z ^ _srl(z, 30)).mul(_s64(_M1))
    z = (z ^ _srl(z, 27)).mul(_s64(_M2))
    return z ^ _srl(z, 31)


def splitmix64_np(idx: np.ndarray, seed: int = IID_SEED) -> np.ndarray:
    """Host twin of splitmix64 (uint64 arithmetic wraps)."""
    with np.errstate(over="ignore"):
        z = (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(_GOLDEN) + np.uint64(seed)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_M2)
        return z ^ (z >> np.uint64(31))


def unigram_cum(text: np.ndarray) -> np.ndarray:
    """Cumulative byte counts of the source text (int64[256])."""
    return np.cumsum(np.bincount(text, minlength=256)).astype(np.int64)


def iid_symbols_np(cum: np.ndarray, start: int, n: int, seed: int = IID_SEED) -> np.ndarray:
    """Symbols start .. start+n-1 of the i.i.d. stream, on the host."""
    T = int(cum[-1])
    r = splitmix64_np(np.arange(start, start + n, dtype=np.uint64), seed) >> np.uint64(32)
    x = ((r * np.uint64(T)) >> np.uint64(32)).astype(np.int64)
    return np.searchsorted(cum, x, side="right").astype(np.uint8)


def code_table(tree, max_len: int = 32) -> tuple[np.ndarray, np.ndarray]:
    """(code bits LSB-first = first branch in bit 0, code length) per byte;
    encode_gpu takes codes of up to 60 bits."""
    code = np.zeros(256, np.int64)
    L = np.zeros(256, np.int64)
    stack = [(0, 0, 0)]
    while stack:
        v, d, c = stack.pop()
        if tree.izero[v] == -1:
            s = tree.sym[v]
            if L[s] == 0:
                L[s], code[s] = d, c
        else:
            stack.append((int(tree.izero[v]), d + 1, c))
            stack.append((int(tree.ione[v]), d + 1, c | (1 << d)))
    if L.max() > max_len:
        raise ValueError(f"codes longer than {max_len} bits")
    return code, L


@dataclass
class IIDStream:
    tree: object            # huffmandecoderongpus_amd.Tree
    data: object            # torch uint8 cuda tensor: payload + pad
    bits: int
    syms: object            # torch uint8 cuda tensor: the symbols encoded

    @property
    def compressed_bytes(self) -> int:
        return (self.bits + 7) // 8

    @property
    def decoded_bytes(self) -> int:
        return int(self.syms.numel())


def encode_gpu(syms, code, lens, device="cuda", chunk: int = 1 << 27):
    """Pack symbols (torch uint8) LSB-first with (code, lens) on the GPU ->
    (payload uint8 tensor with 72 pad bytes, bits).  Codes of distinct
    symbols occupy disjoint bits, so OR is a sum: 32-bit words are built by
    index_add_ of each code's parts in int64 (a code of up to 60 bits spans
    at most three words)."""
    import torch
    codes = torch.as_tensor(code, device=device)
    lt = torch.as_tensor(lens, device=device)
    n = syms.numel()
    total = 0
    offs = []                                   # per-chunk start bits
    for c0 in range(0, n, chunk):
        offs.append(total)
        total += int(lt[syms[c0:c0 + chunk].long()].sum().item())
    nwords = (total + 31) // 32 + 2 + 18        # + pad (72 B)
    words = torch.zeros(nwords, dtype=torch.int64, device=device)
    for i, c0 in enumerate(range(0, n, chunk)):
        s = syms[c0:c0 + chunk].long()
        ln = lt[s]
        pos = torch.cumsum(ln, 0) - ln + offs[i]
        cv = codes[s]
        w, sh = pos >> 5, pos & 31
        words.index_add_(0, w, (cv << sh) & 0xffffffff)
        words.index_add_(0, w + 1, (cv >> (32 - sh)) & 0xffffffff)
        if int(lt.max().item()) > 32:
            words.index_add_(0, w + 2, (cv >> 32) >> (32 - sh))
        del s, ln, pos, cv, w, sh
    payload = words.to(torch.int32).view(torch.uint8)
    return payload, total


def iid_stream(hf, text: np.ndarray, target_bytes: int, device="cuda", seed: int = IID_SEED,
               chunk: int = 1 << 27) -> IIDStream:
    """The i.i.d. stream cut at the last whole symbol within target_bytes of
    payload, encoded on the GPU with hf's codebook."""
    return iid_stream_from(hf.tree(), unigram_cum(text), target_bytes, device, seed, chunk)


def iid_stream_from(tree, cum: np.ndarray, target_bytes: int, device="cuda", seed: int = IID_SEED,
                    chunk: int = 1 << 27) -> IIDStream:
    """i.i.d. symbols with the cumulative counts cum (int64[256], splitmix64
    seed `seed`), cut at the last whole symbol within target_bytes of
    payload, encoded on the GPU with tree's codes."""
    import torch
    code, lens = code_table(tree, 60)
    T = int(cum[-1])
    cum_t = torch.as_tensor(cum, device=device)
    p = np.diff(np.concatenate([[0], cum])) / T
    n = int(8 * target_bytes / float((p * lens).sum()) * 1.01) + 64    # a little more than fits
    syms = torch.empty(n, dtype=torch.uint8, device=device)
    for c0 in range(0, n, chunk):
        c1 = min(c0 + chunk, n)
        r = _srl(splitmix64(torch.arange(c0, c1, dtype=torch.int64, device=device), seed), 32)
        x = (r * T) >> 32
        syms[c0:c1] = torch.searchsorted(cum_t, x, right=True).to(torch.uint8)
        del r, x
    lt = torch.as_tensor(lens, device=device)
    # keep the longest prefix whose bits fit the target
    budget, keep = 8 * target_bytes, 0
    for c0 in range(0, n, chunk):
        cs = torch.cumsum(lt[syms[c0:c0 + chunk].long()], 0)
        k = int(torch.searchsorted(cs, torch.tensor([budget], device=device), right=True).item())
        keep += k
        if k < cs.numel():
            break
        budget -= int(cs[-1].item())
    syms = syms[:keep].clone()
    payload, bits = encode_gpu(syms, code, lens, device, chunk)
    return IIDStream(tree, payload, bits, syms)


# ---------------------------------------------------------------------------
# Byte-alphabet stream: a Huffman code over all 256 byte values (255
# internal nodes, the largest tree a byte alphabet gives -- the state
# machine's 7-bit count steps) for i.i.d. bytes with Zipf-like frequencies.
# ---------------------------------------------------------------------------
BYTE_SEED = 0xB17E5EED
ZIPF_S = 1.1


def byte_counts(seed: int = BYTE_SEED, s: float = ZIPF_S) -> np.ndarray:
    """Counts of the 256 byte values: 2^20 / rank^s (+1), ranks a seeded
    permutation (int64[256], every value present)."""
    rank = np.random.default_rng(seed).permutation(256) + 1
    return (np.floor(float(1 << 20) / rank.astype(np.float64) ** s) + 1).astype(np.int64)


def huffman_tree(counts: np.ndarray):
    """A Huffman code for the symbols with counts > 0, in the reference's
    layout (huffdata.h:12-16: node 0 the root, pre-order, leaves
    izero = ione = -1): deterministic (ties broken by insertion order)."""
    import heapq
    from huffmandecoderongpus_amd import Tree
    heap = [(int(c), i, ("leaf", i)) for i, c in enumerate(counts) if c > 0]
    heapq.heapify(heap)
    k = len(heap)
    if k == 1:
        heap = [(heap[0][0], 0, ("node", heap[0][2], ("leaf", (heap[0][2][1] + 1) & 255)))]
    while len(heap) > 1:
        a = heapq.heappop(heap)
        b = heapq.heappop(heap)
        heapq.heappush(heap, (a[0] + b[0], k, ("node", a[2], b[2])))
        k += 1
    iz, io, sy = [], [], []

    def emit(t):
        v = len(iz)
        iz.append(-1); io.append(-1); sy.append(0)
        if t[0] == "leaf":
            sy[v] = t[1]
        else:
            iz[v] = emit(t[1])
            io[v] = emit(t[2])
        return v
    emit(heap[0][2])
    return Tree(np.array(iz, np.int32), np.array(io, np.int32), np.array(sy, np.uint8))


def byte_stream(target_bytes: int, device="cuda", seed: int = BYTE_SEED, chunk: int = 1 << 27) -> IIDStream:
    """i.i.d. bytes with byte_counts(seed) frequencies, Huffman-coded
    (huffman_tree), cut within target_bytes of payload, encoded on the GPU."""
    counts = byte_counts(seed)
    return iid_stream_from(huffman_tree(counts), np.cumsum(counts).astype(np.int64), target_bytes, device,
                           seed, chunk)
