"""Synthetic workload generators on the CPU (torch CPU tensors): the i.i.d.
variant of SURVEY.md 8d and the packing encoder the GPU runs, checked against
splitmix64's published first output, the numpy twin, the host C encoder and
the oracle decoder."""
import os

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KJV = os.path.join(ROOT, "files", "kjv.txt.huff")


@pytest.fixture(scope="module")
def kjv():
    import huffmandecoderongpus_amd as H
    return H.HuffFile.load(KJV), O.OracleHuff.load(KJV).chain_decode()


def test_splitmix64_known_answer_and_twins():
    import torch
    from huffmandecoderongpus_amd import synth
    # splitmix64 seeded with 0: first output 0xE220A8397B1DCDAF
    assert int(synth.splitmix64_np(np.arange(1), 0)[0]) == 0xE220A8397B1DCDAF
    idx = np.arange(0, 5000, 7)
    a = synth.splitmix64(torch.from_numpy(idx.astype(np.int64))).numpy().view(np.uint64)
    assert np.array_equal(a, synth.splitmix64_np(idx))


def test_iid_symbols_follow_the_unigram(kjv):
    from huffmandecoderongpus_amd import synth
    _, text = kjv
    cum = synth.unigram_cum(text)
    s = synth.iid_symbols_np(cum, 0, 400000)
    p = np.bincount(text, minlength=256) / len(text)
    q = np.bincount(s, minlength=256) / len(s)
    assert set(np.nonzero(q)[0]) <= set(np.nonzero(p)[0])
    assert np.abs(p - q).max() < 0.003


def test_gpu_encoder_matches_host_encoder_and_oracle(kjv):
    from huffmandecoderongpus_amd import synth
    hf, text = kjv
    st = synth.iid_stream(hf, text, 150000, device="cpu", chunk=1 << 15)
    assert st.bits <= 8 * 150000
    syms = st.syms.numpy()
    assert np.array_equal(syms, synth.iid_symbols_np(synth.unigram_cum(text), 0, len(syms)))
    pay, bits = hf.tree().encode(syms)
    nb = (bits + 7) // 8
    assert bits == st.bits
    assert np.array_equal(st.data.numpy()[:nb], pay[:nb])
    h = O.Huff(bits, len(syms), hf.izero, hf.ione, hf.sym, pay[:nb])
    assert np.array_equal(O.OracleHuff.from_arrays(h).chain_decode(), syms)


def test_code_table_matches_code_lengths(kjv):
    from huffmandecoderongpus_amd import synth
    hf, _ = kjv
    code, lens = synth.code_table(hf.tree())
    assert np.array_equal(lens, synth.code_lengths(hf.tree()))
    present = np.nonzero(lens)[0]
    assert len(set((int(code[s]), int(lens[s])) for s in present)) == len(present)


def test_byte_alphabet_huffman_tree():
    """bench's byte-alphabet codebook: a Huffman code over all 256 byte
    values (255 internal nodes), complete (Kraft sum 1), its mean code
    length within a bit of the entropy, and an encode -> oracle decode round
    trip of i.i.d. symbols drawn from its frequencies (host twin of the
    GPU generator)."""
    from huffmandecoderongpus_amd import synth
    counts = synth.byte_counts()
    assert counts.size == 256 and (counts > 0).all()
    t = synth.huffman_tree(counts)
    info = t.info()
    assert info["leaves"] == 256 and info["reachable"] == 511
    code, L = synth.code_table(t, 60)
    assert abs(sum(2.0 ** -int(x) for x in L) - 1.0) < 1e-12
    p = counts / counts.sum()
    H_ = float(-(p * np.log2(p)).sum())
    assert H_ <= float((p * L).sum()) < H_ + 1
    syms = synth.iid_symbols_np(np.cumsum(counts).astype(np.int64), 0, 200000, synth.BYTE_SEED)
    data, bits = t.encode(syms)
    hf = O.Huff(bits, 0, t.izero, t.ione, t.sym, data[: (bits + 7) // 8])
    assert np.array_equal(O.OracleHuff.from_arrays(hf).chain_decode(), syms)
