"""GPU parity of the single-pass decode (hh_one.hip, k_one): byte-exact
against the oracle and the two-pass pipeline (HH_FLAG_TWO_PASS), on the
fixtures, cut streams of random trees (the tail rule, partial tiles), the
kjv-tiled stream, forced column overflows, segments after a prologue,
concurrent decoders on two streams, and the hand-back to the two passes."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

FIXTURES = ["hello", "paper1", "news", "book2", "bible.txt", "world192.txt", "kjv.txt"]


@pytest.fixture(scope="module")
def hh():
    import huffmandecoderongpus_amd as H
    return H


@pytest.fixture(autouse=True)
def single_pass(monkeypatch):
    monkeypatch.setenv("HH_ONE", "1")           # (read when a tree is set)


def _random_tree(rng, nleaves):
    izero, ione, sym = [-1], [-1], [0]
    leaves = [0]
    syms = rng.permutation(256)[:nleaves]
    while len(leaves) < nleaves:
        v = leaves.pop(int(rng.integers(len(leaves))))
        a, b = len(izero), len(izero) + 1
        izero[v], ione[v] = a, b
        izero += [-1, -1]; ione += [-1, -1]; sym += [0, 0]
        leaves += [a, b]
    for k, v in enumerate(leaves):
        sym[v] = int(syms[k])
    return np.array(izero), np.array(ione), np.array(sym), syms


def _oracle(iz, io, sy, data, bits):
    hf = O.Huff(bits, 0, np.asarray(iz, np.int32), np.asarray(io, np.int32),
                np.asarray(sy, np.uint8), np.asarray(data, np.uint8)[: (bits + 7) // 8])
    return O.OracleHuff.from_arrays(hf).chain_decode()


def _dev(data, bits):
    import torch
    buf = np.zeros((bits + 7) // 8 + 64, np.uint8)
    buf[: (bits + 7) // 8] = np.asarray(data, np.uint8)[: (bits + 7) // 8]
    return torch.from_numpy(buf).cuda()


def _decode(hh, dec, d_in, bits, cap):
    import torch
    d_out = torch.full((cap + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    n = dec.decode_device(d_in, bits, d_out)
    torch.cuda.synchronize()
    assert int(d_out[n:n + 64].ne(0xAB).sum()) == 0, "bytes written past the output"
    return d_out[:n].cpu().numpy()


@pytest.mark.parametrize("name", FIXTURES)
def test_single_pass_fixture(hh, files_dir, name):
    """Every variable-length fixture through k_one (state_machine == 2),
    byte-equal to the oracle's chain decode."""
    path = os.path.join(files_dir, name + ".huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec = hh.Decoder(0)
    try:
        dec.set_tree(hf.tree())
        got = _decode(hh, dec, _dev(hf.payload, hf.bits), hf.bits, hf.uncompressedsize)
        st = dec.stats()
        assert st["state_machine"] == 2 and st["exact_fallback"] == 0, st
        assert got.size == ref.size and np.array_equal(got, ref)
    finally:
        dec.close()


@pytest.mark.parametrize("nleaves,seed", [(3, 1), (12, 2), (40, 3), (97, 4), (128, 5), (200, 6), (256, 7)])
def test_single_pass_cut_random_trees(hh, nleaves, seed):
    """Random trees (up to 255 states: 224-bit regions, 5- or 6-bit steps)
    on i.i.d. streams cut mid-code (the tail rule) and at lengths that leave
    a partial last tile, lanes past the end, or a single region.  (3 and 12
    leaves: codes so short that regions overflow the 128-B columns and go
    straight to HBM, one_direct.)"""
    rng = np.random.default_rng(seed)
    iz, io, sy, syms = _random_tree(rng, nleaves)
    p = rng.dirichlet(np.full(nleaves, 0.5))
    t = hh.Tree(iz, io, sy)
    text = rng.choice(syms, size=400_000, p=p).astype(np.uint8)
    data, bits = t.encode(text)
    # (k_one is built for 256- and 224-bit regions: the smaller trees, whose
    # default regions are shorter, are decoded with 256-bit ones; trees of
    # more than 127 states take 224 bits by themselves)
    dec = hh.Decoder(0, lane_bits=256 if nleaves <= 128 else 0)
    try:
        dec.set_tree(t)
        tb = dec.tile_bits()
        assert tb in (64 * 256, 64 * 224), tb
        cuts = sorted({bits, bits - 1, bits // 3 + 7, tb - 1, tb, tb + 1, 5 * tb + 333, 300, 17})
        for cut in cuts:
            if cut <= 0 or cut > bits:
                continue
            ref = _oracle(iz, io, sy, data, cut)
            got = _decode(hh, dec, _dev(data, cut), cut, ref.size + 16)
            st = dec.stats()
            assert st["state_machine"] == 2, (nleaves, cut, st)
            assert got.size == ref.size and np.array_equal(got, ref), (nleaves, cut)
    finally:
        dec.close()


@pytest.mark.parametrize("mib", [64, 1024])
def test_single_pass_tiled_stream_against_two_pass(hh, files_dir, mib):
    """BASELINE configs[2]'s workload: the kjv-tiled stream through k_one
    and through the two passes: both equal the tiled text."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, mib << 20)
    out = torch.full((syn.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
    try:
        for flags, sm in ((0, 2), (hh.FLAG_TWO_PASS, 1)):
            dec = hh.Decoder(0, flags=flags)
            try:
                dec.set_tree(syn.tree)
                out.fill_(0xAB)
                for _ in range(2):                 # (the second: the next epoch's words)
                    n = dec.decode_device(syn.data, syn.bits, out)
                    torch.cuda.synchronize()
                    st = dec.stats()
                    assert st["state_machine"] == sm and st["exact_fallback"] == 0, st
                    assert n == syn.decoded_bytes and synth.verify_tiled(out, syn)
                    assert int(out[n:n + 64].ne(0xAB).sum()) == 0
            finally:
                dec.close()
    finally:
        del out, syn
        torch.cuda.empty_cache()


@pytest.mark.parametrize("capd", ["3", "9"])
def test_single_pass_column_overflow(hh, files_dir, capd, monkeypatch):
    """Columns too small for the regions (HH_ONE_CAPD): the tiles whose runs
    overflow are decoded straight to HBM (one_direct), the others staged --
    the same bytes either way."""
    monkeypatch.setenv("HH_ONE_CAPD", capd)   # read when the tree is set
    for name in ("paper1", "kjv.txt"):
        path = os.path.join(files_dir, name + ".huff")
        hf = hh.HuffFile.load(path)
        ref = O.OracleHuff.load(path).chain_decode()
        dec = hh.Decoder(0)
        try:
            dec.set_tree(hf.tree())
            got = _decode(hh, dec, _dev(hf.payload, hf.bits), hf.bits, hf.uncompressedsize)
            assert dec.stats()["state_machine"] == 2
            assert np.array_equal(got, ref), name
        finally:
            dec.close()


def test_single_pass_segments_match_two_pass(hh, files_dir):
    """Segments (hh_decode_device_range) through k_one against the two
    passes: 5 segments of the kjv-tiled 64 MiB stream, each entered in the
    root after a 2-tile prologue (its entry found by the chain through the
    prologue), give the same lengths, entry and leave states and bytes."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, 64 << 20)
    res = {}
    for flags in (0, hh.FLAG_TWO_PASS):
        dec = hh.Decoder(0, flags=flags)
        try:
            dec.set_tree(syn.tree)
            tb = dec.tile_bits()
            nt = (syn.bits + tb - 1) // tb
            cuts = [0, nt // 5, 2 * nt // 5 + 3, 3 * nt // 5, nt - 1, nt]
            rows = []
            for a, b in zip(cuts[:-1], cuts[1:]):
                pro = min(a, 2)
                t0 = a - pro
                w0 = t0 * tb // 32
                d = syn.data[w0 * 4:]
                out = torch.zeros(((b - t0) * tb) // 2 + 4096, dtype=torch.uint8, device="cuda")
                r = dec.decode_range_ptr(d.data_ptr(), syn.bits - t0 * tb, b - t0, 0, out.data_ptr(),
                                         out.numel(), prologue=pro)
                torch.cuda.synchronize()
                assert dec.stats()["state_machine"] == (1 if flags else 2)
                rows.append((r["out_len"], r["entry_state"], r["leave_state"],
                             out[: r["out_len"]].cpu().numpy().tobytes()))
            res[flags] = rows
        finally:
            dec.close()
    assert res[0] == res[hh.FLAG_TWO_PASS]


def test_single_pass_two_decoders_two_streams(hh, files_dir):
    """Two decoders running k_one at once on two streams (each grid may find
    only part of the chip: its tiles go to its running workgroups in order,
    so neither waits on a workgroup that is not resident), repeated, every
    output checked."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, 256 << 20)
    decs = [hh.Decoder(0), hh.Decoder(0)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.full((syn.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(2)]
    try:
        for d in decs:
            d.set_tree(syn.tree)
        torch.cuda.synchronize()
        for _ in range(3):
            ns = [d.decode_device_async(syn.data, syn.bits, o, s) for d, o, s in zip(decs, outs, streams)]
            for d in decs:
                d.wait()
            torch.cuda.synchronize()
            for n, o, d in zip(ns, outs, decs):
                assert n.value == syn.decoded_bytes and synth.verify_tiled(o, syn)
                assert d.stats()["state_machine"] == 2
            for o in outs:
                o.fill_(0xAB)
    finally:
        for d in decs:
            d.close()
        del outs, syn
        torch.cuda.empty_cache()


def test_single_pass_hand_back_to_two_passes(hh, files_dir, monkeypatch):
    """A single-pass decode that hands itself back (HH_TEST_ONE_RETRY=1, the
    test hook that makes every k_one decode report it; in production: a wait
    that ran out, or more fix rounds than ONE_RMAX) is decoded again by the
    two passes -- synchronously, from hh_decode_host's chunks, and from the
    asynchronous checker while the next decode is queued; every output
    equals the oracle's."""
    import torch
    monkeypatch.setenv("HH_TEST_ONE_RETRY", "1")
    path = os.path.join(files_dir, "kjv.txt.huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec = hh.Decoder(0)
    try:
        dec.set_tree(hf.tree())
        d_in = _dev(hf.payload, hf.bits)
        got = _decode(hh, dec, d_in, hf.bits, hf.uncompressedsize)
        assert dec.stats()["state_machine"] == 1 and np.array_equal(got, ref)
        out = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
        assert np.array_equal(out, ref)
        outs = [torch.full((hf.uncompressedsize + 64,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(3)]
        ns = [dec.decode_device_async(d_in, hf.bits, o) for o in outs]
        dec.wait()
        torch.cuda.synchronize()
        for n, o in zip(ns, outs):
            assert n.value == ref.size and np.array_equal(o[: n.value].cpu().numpy(), ref)
    finally:
        dec.close()
