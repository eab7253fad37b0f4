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
