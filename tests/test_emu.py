"""The fast path's stitching algorithm (hh_algo.h, exactly as the kernel runs
it, tile by tile, on the kernel's transposed LDS layout) emulated on the
host and checked against the oracle.

Covers the reference fixtures at the default and a small region size, random
trees and streams, codes cut off by the end of the stream (the reference's
tail rule), fixed-length codes (region sizes on the code lattice merge at
once) and non-synchronising region sizes (the walks must report failure,
never a wrong answer)."""
import ctypes as C
import os

import numpy as np
import pytest

import huffmandecoderongpus_amd as H
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = os.path.join(ROOT, "files")
EMU = os.path.join(ROOT, "tests", "emu", "libhh_emu.so")
UNSUPPORTED = -10


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(EMU):
        pytest.skip("tests/emu/libhh_emu.so not built (make emu)")
    L = C.CDLL(EMU)
    L.hh_emu_decode.restype = C.c_int64
    L.hh_emu_decode.argtypes = [C.c_void_p] * 3 + [C.c_int32, C.c_void_p, C.c_uint64,
                                                   C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p]
    return L


def run_emu(emu, izero, ione, sym, data, bits, S):
    iz = np.ascontiguousarray(izero, np.int32)
    io = np.ascontiguousarray(ione, np.int32)
    sy = np.ascontiguousarray(sym, np.uint8)
    d = np.zeros((bits + 7) // 8 + 64, np.uint8)
    d[: (bits + 7) // 8] = np.asarray(data, np.uint8)[: (bits + 7) // 8]
    out = np.zeros(bits + 16, np.uint8)
    st = np.zeros(8, np.int64)
    n = emu.hh_emu_decode(iz.ctypes.data, io.ctypes.data, sy.ctypes.data, len(iz), d.ctypes.data,
                          bits, S, out.ctypes.data, len(out), st.ctypes.data)
    return n, out[: max(n, 0)], st


def oracle_chain(izero, ione, sym, data, bits):
    hf = O.Huff(bits, 0, np.asarray(izero, np.int32), np.asarray(ione, np.int32),
                np.asarray(sym, np.uint8), np.asarray(data, np.uint8)[: (bits + 7) // 8])
    return O.OracleHuff.from_arrays(hf).chain_decode()


@pytest.mark.parametrize("name", ["hello", "paper1", "news", "book2", "kjv.txt", "E.coli",
                                  "world192.txt", "bible.txt"])
@pytest.mark.parametrize("S", [0, 96])
def test_fixtures(emu, name, S):
    hf = H.HuffFile.load(os.path.join(FILES, name + ".huff"))
    ref = O.OracleHuff.load(os.path.join(FILES, name + ".huff")).chain_decode()
    n, out, st = run_emu(emu, hf.izero, hf.ione, hf.sym, hf.payload, hf.bits, S)
    if S and n == UNSUPPORTED:    # small regions: runs longer than HH_KM regions
        assert st[2] > 0          # are detected, never mis-decoded
        return
    assert n == len(ref) and np.array_equal(out, ref), (n, st)


def random_tree(rng, nleaves):
    """Random full binary tree in the reference's node layout (root = 0)."""
    izero, ione, sym = [-1], [-1], [0]
    leaves = [0]
    syms = rng.permutation(256)[:nleaves]
    while len(leaves) < nleaves:
        v = leaves.pop(int(rng.integers(len(leaves))))
        a, b = len(izero), len(izero) + 1
        izero[v], ione[v] = a, b
        sym[v] = int(rng.integers(256))          # internal nodes carry a byte too
        izero += [-1, -1]; ione += [-1, -1]; sym += [0, 0]
        leaves += [a, b]
    for k, v in enumerate(leaves):
        sym[v] = int(syms[k])
    return np.array(izero), np.array(ione), np.array(sym), syms


@pytest.mark.parametrize("seed", range(12))
def test_random_trees_and_tails(emu, seed):
    rng = np.random.default_rng(seed)
    nleaves = int(rng.integers(2, 120))
    iz, io, sy, syms = random_tree(rng, nleaves)
    t = H.Tree(iz, io, sy)
    if t.info()["maxlen"] > 64:
        pytest.skip("encoder limit")
    p = rng.dirichlet(np.full(nleaves, 0.3))
    text = rng.choice(syms, size=int(rng.integers(1, 60000)), p=p).astype(np.uint8)
    data, bits = t.encode(text)
    for cut in (bits, bits - 1, max(1, bits // 3 + 1)):   # cut codes exercise the tail rule
        ref = oracle_chain(iz, io, sy, data, cut)
        g = t.info()["len_gcd"]
        for S in (0, 64 if 64 % g == 0 else 0):
            n, out, st = run_emu(emu, iz, io, sy, data, cut, S)
            if n == UNSUPPORTED:
                assert st[2] > 0
                continue
            assert n == len(ref), (cut, S)
            assert np.array_equal(out, ref), (cut, S)


def test_empty_stream(emu):
    hf = H.HuffFile.load(os.path.join(FILES, "hello.huff"))
    n, out, st = run_emu(emu, hf.izero, hf.ione, hf.sym, hf.payload, 0, 0)
    assert n == 0


def complete_tree(depth):
    iz, io, sy = [-1], [-1], [0]
    frontier = [0]
    for _ in range(depth):
        nxt = []
        for v in frontier:
            a, b = len(iz), len(iz) + 1
            iz[v], io[v] = a, b
            iz += [-1, -1]; io += [-1, -1]; sy += [0, 0]
            nxt += [a, b]
        frontier = nxt
    for k, v in enumerate(frontier):
        sy[v] = k & 255
    return np.array(iz), np.array(io), np.array(sy)


def test_fixed_length_code_on_the_lattice(emu):
    """5-bit fixed-length code: the default region size is a multiple of 5
    (160 bits), so every region starts on a code boundary and every walk
    merges at once."""
    iz, io, sy = complete_tree(5)
    rng = np.random.default_rng(1)
    bits = 5 * 40000
    data = rng.integers(0, 256, size=bits // 8 + 1).astype(np.uint8)
    ref = oracle_chain(iz, io, sy, data, bits)
    n, out, st = run_emu(emu, iz, io, sy, data, bits, 0)
    assert st[3] % 5 == 0 and st[3] % 32 == 0
    assert n == len(ref) == 40000 and np.array_equal(out, ref)
    assert st[1] == 0


def test_fixed_length_code_off_the_lattice_multi_region_walks(emu):
    """The same 5-bit code with 256-bit regions: region starts drift by one
    bit per region against the code lattice, so walks cross up to 5 regions
    before they merge (covered regions, k > 1) -- and the tiles' leaving
    state is the entering one shifted, exercising the transfer tables."""
    iz, io, sy = complete_tree(5)
    rng = np.random.default_rng(3)
    bits = 5 * 100000
    data = rng.integers(0, 256, size=bits // 8 + 1).astype(np.uint8)
    ref = oracle_chain(iz, io, sy, data, bits)
    n, out, st = run_emu(emu, iz, io, sy, data, bits, 256)
    assert n == len(ref) == 100000 and np.array_equal(out, ref)
    assert st[4] == 5 and st[1] > 0


def test_non_synchronising_code_is_detected(emu):
    """An 11-bit fixed-length code realigns with 96-bit regions only every
    11 regions (> HH_KM): the walks must fail (-> exact path), never
    mis-decode; the default region size (352 = lcm(32, 11)) aligns at once."""
    iz, io, sy = complete_tree(11)
    rng = np.random.default_rng(2)
    bits = 11 * 30000
    data = rng.integers(0, 256, size=bits // 8 + 1).astype(np.uint8)
    ref = oracle_chain(iz, io, sy, data, bits)
    n, out, st = run_emu(emu, iz, io, sy, data, bits, 96)
    assert n == UNSUPPORTED and st[2] > 0
    n, out, st = run_emu(emu, iz, io, sy, data, bits, 0)
    assert st[3] == 352
    assert n == len(ref) and np.array_equal(out, ref)


# ---------------------------------------------------------------------------
# The state-machine decode (round 3's main path, hh_fsm.hip), emulated tile
# by tile with the kernels' tables and per-lane rules (tests/emu/hh_fsm_emu.cpp)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def femu():
    if not os.path.exists(EMU):
        pytest.skip("tests/emu/libhh_emu.so not built (make emu)")
    L = C.CDLL(EMU)
    L.hh_fsm_emu_decode.restype = C.c_int64
    L.hh_fsm_emu_decode.argtypes = [C.c_void_p] * 3 + [C.c_int32, C.c_void_p, C.c_uint64, C.c_uint32,
                                                       C.c_int32, C.c_uint64, C.c_uint64, C.c_uint32,
                                                       C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                                       C.c_void_p]
    L.hh_fsm_emu_tables.restype = C.c_int64
    L.hh_fsm_emu_tables.argtypes = [C.c_void_p] * 3 + [C.c_int32, C.c_uint32, C.c_void_p]
    L.hh_fsm_emu_set_k.restype = None
    L.hh_fsm_emu_set_k.argtypes = [C.c_uint32]
    L.hh_fsm_emu_set_m.restype = None
    L.hh_fsm_emu_set_m.argtypes = [C.c_uint32]
    return L


def run_femu(L, izero, ione, sym, data, bits, S=0, G=-1, ntiles=0, prologue=0, in_state=0, K=0, M=1):
    L.hh_fsm_emu_set_k(K)                     # emission step bits (0: the default, 6)
    L.hh_fsm_emu_set_m(M)                     # regions per lane of the count pass
    iz = np.ascontiguousarray(izero, np.int32)
    io = np.ascontiguousarray(ione, np.int32)
    sy = np.ascontiguousarray(sym, np.uint8)
    d = np.zeros((bits + 7) // 8 + 64, np.uint8)
    d[: (bits + 7) // 8] = np.asarray(data, np.uint8)[: (bits + 7) // 8]
    out = np.zeros(bits + 16, np.uint8)
    st = np.zeros(9, np.int64)
    lv, en = C.c_uint32(), C.c_uint32()
    n = L.hh_fsm_emu_decode(iz.ctypes.data, io.ctypes.data, sy.ctypes.data, len(iz), d.ctypes.data, bits, S, G,
                            ntiles, prologue, in_state, out.ctypes.data, len(out), st.ctypes.data,
                            C.byref(lv), C.byref(en))
    return n, out[: max(n, 0)], st, lv.value, en.value


@pytest.mark.parametrize("name", ["hello", "paper1", "news", "book2", "kjv.txt", "E.coli",
                                  "world192.txt", "bible.txt"])
@pytest.mark.parametrize("S,K", [(0, 6), (96, 6), (0, 7), (96, 7)])
def test_fsm_fixtures(femu, name, S, K):
    """Every fixture, 6- and 7-bit emission steps (7 with 256-bit regions: a
    4-bit remainder step; with 96: a 5-bit one)."""
    hf = H.HuffFile.load(os.path.join(FILES, name + ".huff"))
    ref = O.OracleHuff.load(os.path.join(FILES, name + ".huff")).chain_decode()
    n, out, st, _, _ = run_femu(femu, hf.izero, hf.ione, hf.sym, hf.payload, hf.bits, S, K=K)
    assert n == len(ref) and np.array_equal(out, ref), (n, st)


def test_fsm_walks_that_meet_late_are_exact(femu):
    """Small regions and heads make guesses miss often and walks run past
    their region (the rounds of walks, the next tile's corrections over
    several regions): kjv.txt with 64-bit regions and 8-bit heads."""
    hf = H.HuffFile.load(os.path.join(FILES, "kjv.txt.huff"))
    ref = O.OracleHuff.load(os.path.join(FILES, "kjv.txt.huff")).chain_decode()
    n, out, st, _, _ = run_femu(femu, hf.izero, hf.ione, hf.sym, hf.payload, hf.bits, 64, 8)
    assert n == len(ref) and np.array_equal(out, ref)
    assert st[2] > 0 and st[6] > 0           # walks past their region; multi-region corrections


@pytest.mark.parametrize("M", [2, 4, 8])
def test_fsm_lanes_of_several_regions(femu, M):
    """The count pass with M consecutive regions per lane (a head guesses
    only a lane's first region; the chain is carried through the others):
    every fixture, and kjv.txt with small regions and short heads so that
    walks cross several regions of a lane and the next tile's corrections
    span lanes."""
    try:
        _lanes_of_several_regions(femu, M)
    finally:
        femu.hh_fsm_emu_set_m(1)              # (the library's setting outlives the test)


def _lanes_of_several_regions(femu, M):
    for name in ("hello", "paper1", "kjv.txt", "E.coli", "world192.txt"):
        hf = H.HuffFile.load(os.path.join(FILES, name + ".huff"))
        ref = O.OracleHuff.load(os.path.join(FILES, name + ".huff")).chain_decode()
        n, out, st, _, _ = run_femu(femu, hf.izero, hf.ione, hf.sym, hf.payload, hf.bits, M=M)
        assert n == len(ref) and np.array_equal(out, ref), (name, n, st)
    hf = H.HuffFile.load(os.path.join(FILES, "kjv.txt.huff"))
    ref = O.OracleHuff.load(os.path.join(FILES, "kjv.txt.huff")).chain_decode()
    n, out, st, _, _ = run_femu(femu, hf.izero, hf.ione, hf.sym, hf.payload, hf.bits, 64, 8, M=M)
    assert n == len(ref) and np.array_equal(out, ref)
    assert st[2] > 0 and st[6] > 0
    rng = np.random.default_rng(40 + M)
    for _ in range(4):
        nleaves = int(rng.integers(2, 120))
        iz, io, sy, syms = random_tree(rng, nleaves)
        t = H.Tree(iz, io, sy)
        if t.info()["maxlen"] > 64:
            continue
        text = rng.choice(syms, size=int(rng.integers(1, 200000)), p=rng.dirichlet(np.full(nleaves, 0.3))).astype(np.uint8)
        data, bits = t.encode(text)
        for cut in (bits, bits - 1, max(1, bits // 3 + 1)):
            ref = oracle_chain(iz, io, sy, data, cut)
            n, out, st, _, _ = run_femu(femu, iz, io, sy, data, cut, M=M)
            if n == UNSUPPORTED:
                continue
            assert n == len(ref) and np.array_equal(out, ref), (cut, st)


@pytest.mark.parametrize("seed", range(12))
def test_fsm_random_trees_and_tails(femu, seed):
    rng = np.random.default_rng(seed)
    nleaves = int(rng.integers(2, 120))
    iz, io, sy, syms = random_tree(rng, nleaves)
    t = H.Tree(iz, io, sy)
    if t.info()["maxlen"] > 64:
        pytest.skip("encoder limit")
    p = rng.dirichlet(np.full(nleaves, 0.3))
    text = rng.choice(syms, size=int(rng.integers(1, 60000)), p=p).astype(np.uint8)
    data, bits = t.encode(text)
    for cut in (bits, bits - 1, max(1, bits // 3 + 1)):   # cut codes exercise the tail rule
        ref = oracle_chain(iz, io, sy, data, cut)
        for S, K in ((0, 6), (64, 6), (0, 7)):
            n, out, st, _, _ = run_femu(femu, iz, io, sy, data, cut, S, K=K)
            if n == UNSUPPORTED:       # a code whose chains never meet (lattice)
                continue
            assert n == len(ref) and np.array_equal(out, ref), (cut, S, K, st)


def test_fsm_long_codes(femu):
    """Codes of up to 40 bits (a skewed tree): the state machine has no code
    length limit (round 2's fast path stopped at 32 bits)."""
    iz, io, sy = [-1], [-1], [0]
    v = 0
    for depth in range(40):                  # a caterpillar: code lengths 1..40
        a, b = len(iz), len(iz) + 1
        iz[v], io[v] = a, b
        iz += [-1, -1]; io += [-1, -1]; sy += [depth & 255, (depth + 100) & 255]
        v = b
    iz, io, sy = np.array(iz), np.array(io), np.array(sy)
    t = H.Tree(iz, io, sy)
    assert t.info()["maxlen"] == 40
    rng = np.random.default_rng(7)
    leaves = [i for i in range(len(iz)) if iz[i] == -1]
    text = sy[rng.choice(leaves, size=20000, p=np.full(len(leaves), 1 / len(leaves)))].astype(np.uint8)
    data, bits = t.encode(text)
    ref = oracle_chain(iz, io, sy, data, bits)
    n, out, st, _, _ = run_femu(femu, iz, io, sy, data, bits)
    assert n == len(ref) and np.array_equal(out, ref)


def test_fsm_segments_concatenate(femu):
    """Segments (multi-GPU shards): tiles [a, b) decoded with PROBE tiles of
    the predecessor as a prologue; each entry equals the predecessor's leave
    state and the outputs concatenate to the stream."""
    hf = H.HuffFile.load(os.path.join(FILES, "kjv.txt.huff"))
    ref = O.OracleHuff.load(os.path.join(FILES, "kjv.txt.huff")).chain_decode()
    n, _, st, _, _ = run_femu(femu, hf.izero, hf.ione, hf.sym, hf.payload, hf.bits)
    tb = 64 * int(st[3])
    nt = (hf.bits + tb - 1) // tb
    cuts = [0, nt // 5, nt // 2, nt - 3, nt]
    parts, prev_leave = [], 0
    payload = np.asarray(hf.payload, np.uint8)
    for a, b in zip(cuts, cuts[1:]):
        pro = min(2, a)
        start = (a - pro) * tb
        sub = payload[start // 8:]
        bits = min(hf.bits - start, (b - a + pro + 1) * tb)
        m, out, _, leave, entry = run_femu(femu, hf.izero, hf.ione, hf.sym, sub, bits, ntiles=b - a + pro,
                                           prologue=pro)
        assert m >= 0
        assert entry == prev_leave          # the prologue found the true entry state
        parts.append(out)
        prev_leave = leave
    got = np.concatenate(parts)
    assert len(got) == len(ref) and np.array_equal(got, ref)


def test_fsm_fixed_length_codes(femu):
    """Fixed-length codes: regions on the code lattice need no head (the root
    is always right); off the lattice (S not a multiple of L) chains never
    meet and the decode reports it (-> the segment path), never a wrong
    answer."""
    for L_, S in ((5, 0), (3, 0), (5, 256)):
        iz, io, sy = complete_tree(L_)
        rng = np.random.default_rng(L_)
        bits = L_ * 30000
        data = rng.integers(0, 256, size=bits // 8 + 1).astype(np.uint8)
        ref = oracle_chain(iz, io, sy, data, bits)
        n, out, st, _, _ = run_femu(femu, iz, io, sy, data, bits, S)
        if S and S % L_:
            assert n == UNSUPPORTED
        else:
            assert st[4] == 0 and st[1] == 0     # no head, no walks
            assert n == len(ref) and np.array_equal(out, ref)


def test_fsm_tables_shape(femu):
    """State machine sizes of the fixtures: emission steps of 6 bits for codes
    of >= 2 bits, a 4-bit remainder step for 256-bit regions."""
    hf = H.HuffFile.load(os.path.join(FILES, "kjv.txt.huff"))
    info = np.zeros(5, np.uint32)
    iz = np.ascontiguousarray(hf.izero, np.int32)
    io = np.ascontiguousarray(hf.ione, np.int32)
    sy = np.ascontiguousarray(hf.sym, np.uint8)
    assert femu.hh_fsm_emu_tables(iz.ctypes.data, io.ctypes.data, sy.ctypes.data, len(iz), 256,
                                  info.ctypes.data) == 0
    assert list(info) == [83, 6, 4, 128, 8]
    femu.hh_fsm_emu_set_k(7)
    try:
        assert femu.hh_fsm_emu_tables(iz.ctypes.data, io.ctypes.data, sy.ctypes.data, len(iz), 256,
                                      info.ctypes.data) == 0
    finally:
        femu.hh_fsm_emu_set_k(0)
    assert list(info) == [83, 7, 4, 128, 8]
    # a byte alphabet (256 leaves, 255 states): 7-bit count steps over
    # 224-bit regions (an entry's 16 bits hold an 8-bit state's row), 6-bit
    # emission steps whatever is asked (the et row field), 126-bit heads
    rng = np.random.default_rng(5)
    iz, io, sy, _ = random_tree(rng, 256)
    iz, io, sy = (np.ascontiguousarray(a, t) for a, t in ((iz, np.int32), (io, np.int32), (sy, np.uint8)))
    for K in (0, 7):
        femu.hh_fsm_emu_set_k(K)
        try:
            assert femu.hh_fsm_emu_tables(iz.ctypes.data, io.ctypes.data, sy.ctypes.data, len(iz), 0,
                                          info.ctypes.data) == 0
        finally:
            femu.hh_fsm_emu_set_k(0)
        assert list(info) == [255, 6, 224 % 6, 126, 7]


@pytest.mark.parametrize("seed", range(8))
def test_fsm_byte_alphabet_trees(femu, seed):
    """Trees of 129..256 leaves (128..255 states, more than 8-bit count steps
    can number): 7-bit count steps over 224-bit regions, streams cut inside
    codes (tail rule), 6- and 7-bit emission asked for, against the
    oracle."""
    rng = np.random.default_rng(1000 + seed)
    nleaves = int(rng.integers(129, 257))
    iz, io, sy, syms = random_tree(rng, nleaves)
    t = H.Tree(iz, io, sy)
    if t.info()["maxlen"] > 64:
        pytest.skip("encoder limit")
    p = rng.dirichlet(np.full(nleaves, 0.3))
    text = rng.choice(syms, size=int(rng.integers(30000, 120000)), p=p).astype(np.uint8)
    data, bits = t.encode(text)
    for cut in (bits, bits - 1, max(1, bits // 3 + 1), 14336 * 2 + 5):
        cut = min(cut, bits)
        ref = oracle_chain(iz, io, sy, data, cut)
        for K in (0, 7):
            n, out, st, _, _ = run_femu(femu, iz, io, sy, data, cut, K=K)
            assert st[3] == 224 and st[4] % 7 == 0, st
            assert n == len(ref) and np.array_equal(out, ref), (cut, K, st)
