"""The device encoder (hh_encode_device, csrc/hh_encode.hip; SURVEY.md 8(f)
rank 4): byte-identical to the host encoder hh_encode on random trees,
the shipped fixtures' trees and the byte alphabet, at sizes on and off its
4096-symbol chunk boundaries, and decoded back by the oracle and by the
GPU decoder (round trips).  Errors: a symbol absent from the tree, too
small an output buffer."""

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hh():
    import huffmandecoderongpus_amd as H
    return H


def _random_tree(rng, nleaves):
    izero, ione, sym = [-1], [-1], [0]
    leaves = [0]
    syms = rng.permutation(256)[:nleaves]
    while len(leaves) < nleaves:
        v = leaves.pop(int(rng.integers(len(leaves))))
        a, b = len(izero), len(izero) + 1
        izero[v], ione[v] = a, b
        sym[v] = int(rng.integers(256))
        izero += [-1, -1]; ione += [-1, -1]; sym += [0, 0]
        leaves += [a, b]
    for k, v in enumerate(leaves):
        sym[v] = int(syms[k])
    return np.array(izero), np.array(ione), np.array(sym), syms


def _encode_both(hh, tree, syms):
    """(host bytes, host bits, device bytes, device bits)."""
    import torch
    host, hbits = tree.encode(syms)
    nb = (hbits + 7) // 8
    d_syms = torch.from_numpy(np.ascontiguousarray(syms, np.uint8)).cuda()
    cap = (hbits + 31) // 32 * 4 + hh.PAYLOAD_PAD
    out = torch.full((cap,), 0xAB, dtype=torch.uint8, device="cuda")
    dbits = hh.encode_device(tree, d_syms, out)
    torch.cuda.synchronize()
    dev = out.cpu().numpy()
    # nothing written past the stream's last 32-bit word
    assert (dev[(dbits + 31) // 32 * 4:] == 0xAB).all()
    return host[:nb], hbits, dev[:nb], dbits


@pytest.mark.parametrize("nleaves,n", [(2, 1), (5, 4095), (40, 4096), (40, 4097), (129, 100_003),
                                       (256, 1_000_001)])
def test_encode_device_matches_host(hh, nleaves, n):
    rng = np.random.default_rng(nleaves * 7 + n)
    iz, io, sy, syms = _random_tree(rng, nleaves)
    p = rng.dirichlet(np.full(nleaves, 0.5))
    text = rng.choice(syms, size=n, p=p).astype(np.uint8)
    tree = hh.Tree(iz, io, sy)
    host, hbits, dev, dbits = _encode_both(hh, tree, text)
    assert dbits == hbits
    assert np.array_equal(dev, host)
    # the oracle decodes it back
    hf = O.Huff(dbits, 0, np.asarray(iz, np.int32), np.asarray(io, np.int32), np.asarray(sy, np.uint8), dev)
    back = O.OracleHuff.from_arrays(hf).chain_decode()
    assert np.array_equal(back, text)


@pytest.mark.parametrize("name", ["paper1", "kjv.txt", "E.coli"])
def test_encode_device_fixture_round_trip(hh, files_dir, name):
    """A fixture's text, re-encoded on the GPU with its own tree, is its
    payload bit for bit; the GPU decoder decodes the re-encoded stream of the
    text tiled to 64 MiB."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir, name)
    tree = hf.tree()
    host, hbits, dev, dbits = _encode_both(hh, tree, text)
    assert dbits == hf.bits
    # (the file's last byte may carry bits past the stream: compare the stream's)
    pay = np.array(hf.payload, np.uint8)
    if hf.bits % 8:
        pay[-1] &= (1 << (hf.bits % 8)) - 1
    assert np.array_equal(dev, pay)
    # tiled to 64 MiB of symbols: encode on the GPU, decode on the GPU
    reps = (64 << 20) // len(text) + 1
    d_syms = torch.from_numpy(np.ascontiguousarray(text)).cuda().repeat(reps)[: 64 << 20]
    out = torch.zeros((d_syms.numel() * 24 + 31) // 32 * 4 + hh.PAYLOAD_PAD, dtype=torch.uint8, device="cuda")
    bits = hh.encode_device(tree, d_syms, out)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(tree)
        got = torch.empty(d_syms.numel() + 4096, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(out, bits, got)
        torch.cuda.synchronize()
        assert n == d_syms.numel() and torch.equal(got[:n], d_syms)
    finally:
        dec.close()


def test_encode_device_byte_alphabet(hh):
    """bench's byte-alphabet code (256 leaves): the GPU encoder against
    synth's torch-op encoder on the same symbols."""
    import torch
    from huffmandecoderongpus_amd import synth
    byt = synth.byte_stream(8 << 20)
    out = torch.zeros(byt.compressed_bytes + 64, dtype=torch.uint8, device="cuda")
    bits = hh.encode_device(byt.tree, byt.syms, out)
    torch.cuda.synchronize()
    assert bits == byt.bits
    nb = (bits + 7) // 8
    assert torch.equal(out[:nb], byt.data[:nb])


def test_encode_device_errors(hh):
    import torch
    rng = np.random.default_rng(5)
    iz, io, sy, syms = _random_tree(rng, 10)
    tree = hh.Tree(iz, io, sy)
    absent = next(v for v in range(256) if v not in set(int(x) for x in syms))
    d = torch.from_numpy(np.array(list(syms) * 100 + [absent], np.uint8)).cuda()
    out = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(hh.HipHuffError):
        hh.encode_device(tree, d, out)
    d = torch.from_numpy(np.array(list(syms) * 100, np.uint8)).cuda()
    with pytest.raises(hh.HipHuffError):
        hh.encode_device(tree, d, out[:8])
    assert hh.encode_device(tree, d[:0], out) == 0


def test_two_encoders_two_streams(hh):
    """Encoders with their own workspaces (hh_encoder_*):
    two threads, each with an encoder and a stream, encode different trees'
    streams at once -- repeatedly, with growing sizes (workspace growth
    without a device-wide wait) -- each byte-identical to the host encoder."""
    import threading
    import torch
    rng = np.random.default_rng(123)
    jobs = []
    for k, nleaves in enumerate((40, 200)):
        iz, io, sy, syms = _random_tree(rng, nleaves)
        tree = hh.Tree(iz, io, sy)
        text = rng.choice(syms, size=3_000_000 + 77777 * k).astype(np.uint8)
        jobs.append((tree, text))
    errs = []

    def work(k):
        try:
            tree, text = jobs[k]
            enc = hh.Encoder(0)
            st = torch.cuda.Stream()
            for n in (100_000, 1_000_003, text.size):
                ref, rbits = tree.encode(text[:n])
                d_syms = torch.from_numpy(text[:n]).cuda()
                cap = (rbits + 31) // 32 * 4 + 64
                out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                bits = enc.encode(tree, d_syms, out, st)
                st.synchronize()
                got = out[: (bits + 7) // 8].cpu().numpy()
                if bits != rbits or not np.array_equal(got, ref[: (rbits + 7) // 8]):
                    errs.append((k, n, bits, rbits))
            enc.close()
        except Exception as e:                        # (reported by the main thread)
            errs.append((k, repr(e)))

    ts = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
