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
