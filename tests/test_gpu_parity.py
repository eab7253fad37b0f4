"""GPU parity: the HIP path vs the oracle, byte-exact (bit-exact integer work)."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

FIXTURES = ["hello", "paper1", "news", "book2", "bible.txt", "world192.txt", "kjv.txt", "E.coli"]


@pytest.fixture(scope="module")
def hh():
    import huffmandecoderongpus_amd as H
    return H


@pytest.fixture(scope="module")
def dec(hh):
    d = hh.Decoder(0)
    yield d
    d.close()


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_host(hh, dec, files_dir, name):
    path = os.path.join(files_dir, name + ".huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec.set_tree(hf.tree())
    out = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
    st = dec.stats()
    assert st["exact_fallback"] == 0
    assert st["state_machine"] in (1, 2) or st["fixed_length"] == 1     # (E.coli: k_fixed)
    assert len(out) == len(ref) == hf.uncompressedsize
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_device(hh, dec, files_dir, name):
    import torch
    path = os.path.join(files_dir, name + ".huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec.set_tree(hf.tree())
    d_in = torch.from_numpy(hf.data.copy()).cuda()
    d_out = torch.zeros(hf.uncompressedsize + 64, dtype=torch.uint8, device="cuda")
    n = dec.decode_device(d_in, hf.bits, d_out)
    torch.cuda.synchronize()
    assert dec.stats()["exact_fallback"] == 0      # the fast path decoded it
    assert dec.stats()["state_machine"] in (1, 2) or dec.stats()["fixed_length"] == 1
    assert n == len(ref)
    assert np.array_equal(d_out[:n].cpu().numpy(), ref)
    assert int(d_out[n:].sum().item()) == 0   # nothing written past the end


@pytest.mark.parametrize("name", ["hello", "paper1", "news", "E.coli"])
def test_stage_pipeline(hh, dec, files_dir, name):
    import torch
    path = os.path.join(files_dir, name + ".huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec.set_tree(hf.tree())
    d_in = torch.from_numpy(hf.data.copy()).cuda()
    d_out = torch.zeros(hf.bits + 1, dtype=torch.uint8, device="cuda")
    n = dec.stage_pipeline_ptr(d_in.data_ptr(), hf.bits, d_out.data_ptr(), d_out.numel())
    torch.cuda.synchronize()
    assert n == len(ref)
    assert np.array_equal(d_out[:n].cpu().numpy(), ref)


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


def _complete_tree(depth):
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


def _oracle(iz, io, sy, data, bits):
    hf = O.Huff(bits, 0, np.asarray(iz, np.int32), np.asarray(io, np.int32),
                np.asarray(sy, np.uint8), np.asarray(data, np.uint8)[: (bits + 7) // 8])
    return O.OracleHuff.from_arrays(hf).chain_decode()


def _decode_dev(hh, dec, data, bits, cap):
    import torch
    buf = np.zeros((bits + 7) // 8 + 64, np.uint8)
    buf[: (bits + 7) // 8] = np.asarray(data, np.uint8)[: (bits + 7) // 8]
    d_in = torch.from_numpy(buf).cuda()
    d_out = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
    n = dec.decode_device(d_in, bits, d_out)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    assert int(out[n:].astype(np.int64).sum()) == 0, "bytes written past the output"
    return out[:n]


@pytest.mark.parametrize("seed", range(6))
def test_random_trees_and_cut_streams(hh, seed):
    """Random codes and streams (multi-tile), cut at arbitrary bits: the
    reference's tail rule for a code cut off by the end of the stream."""
    rng = np.random.default_rng(100 + seed)
    nleaves = int(rng.integers(2, 150))
    iz, io, sy, syms = _random_tree(rng, nleaves)
    t = hh.Tree(iz, io, sy)
    if t.info()["maxlen"] > 60:
        pytest.skip("encoder limit")
    p = rng.dirichlet(np.full(nleaves, 0.3))
    text = rng.choice(syms, size=int(rng.integers(200000, 900000)), p=p).astype(np.uint8)
    data, bits = t.encode(text)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(t)
        for cut in (bits, bits - 1, bits // 3 + 7):
            ref = _oracle(iz, io, sy, data, cut)
            got = _decode_dev(hh, dec, data, cut, cut + 16)
            assert len(got) == len(ref) and np.array_equal(got, ref), cut
            assert dec.stats()["exact_fallback"] == 0
    finally:
        dec.close()


def test_multi_region_walks_and_transfer_tables(hh):
    """5-bit fixed-length code with 256-bit regions: region starts drift one
    bit per region against the code lattice, so walks cover up to 4 regions
    and tiles leave non-CONST states (look-back through the tables)."""
    iz, io, sy = _complete_tree(5)
    rng = np.random.default_rng(7)
    bits = 5 * 600000
    data = rng.integers(0, 256, size=bits // 8 + 1).astype(np.uint8)
    ref = _oracle(iz, io, sy, data, bits)
    dec = hh.Decoder(0, lane_bits=256)
    try:
        dec.set_tree(hh.Tree(iz, io, sy))
        got = _decode_dev(hh, dec, data, bits, bits)
        assert dec.stats()["exact_fallback"] == 0
        assert len(got) == len(ref) and np.array_equal(got, ref)
    finally:
        dec.close()


@pytest.mark.parametrize("depth", range(1, 9))
def test_fixed_length_codes_unpacked(hh, depth):
    """Complete fixed-length codes (2^L symbols of L bits: E.coli's shape)
    are unpacked by k_fixed; streams cut inside a code take the tail rule.
    Both paths -- k_fixed and the general pipeline (HH_FLAG_NO_FIXED = 4) --
    against the oracle, on an unaligned output too."""
    import torch
    rng = np.random.default_rng(depth)
    iz, io, sy = _complete_tree(depth)
    sy = sy.copy()
    sy[iz >= 0] = rng.integers(0, 256, int((iz >= 0).sum()))   # internal nodes: tail-rule bytes
    tree = hh.Tree(iz, io, sy)
    for bits in (1, depth, 16 * depth + 1, 100003, (1 << 20) * depth + depth - 1):
        data = rng.integers(0, 256, (bits + 7) // 8 + 8, dtype=np.uint8)
        want = _oracle(iz, io, sy, data, bits)
        for flags in (0, 4):
            dec = hh.Decoder(0, flags=flags)
            try:
                dec.set_tree(tree)
                got = _decode_dev(hh, dec, data, bits, len(want) + 16)
                assert dec.stats()["fixed_length"] == (1 if flags == 0 else 0)
            finally:
                dec.close()
            assert len(got) == len(want) and np.array_equal(got, want), (depth, bits, flags)
    # an output pointer off 16-B alignment
    bits = 4096 * depth + 1
    data = rng.integers(0, 256, (bits + 7) // 8 + 8, dtype=np.uint8)
    want = _oracle(iz, io, sy, data, bits)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(tree)
        buf = np.zeros((bits + 7) // 8 + 64, np.uint8)
        buf[: (bits + 7) // 8] = data[: (bits + 7) // 8]
        d_in = torch.from_numpy(buf).cuda()
        d_out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(d_in, bits, d_out[3:])
        torch.cuda.synchronize()
        got = d_out.cpu().numpy()
        assert n == len(want) and np.array_equal(got[3:3 + n], want)
        assert not got[:3].any() and not got[3 + n:].any()
    finally:
        dec.close()


def test_capacity_error(hh, files_dir):
    path = os.path.join(files_dir, "paper1.huff")
    hf = hh.HuffFile.load(path)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(hf.tree())
        with pytest.raises(hh.HipHuffError):
            dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize - 1)
    finally:
        dec.close()


@pytest.mark.parametrize("src,mib", [("kjv.txt", 64), ("kjv.txt", 1024), ("E.coli", 1024)])
def test_synthetic_full_size(hh, files_dir, src, mib):
    """BASELINE.json's workload size (1 GiB compressed): kjv.txt tiled and
    encoded with its own codebook must decode to the tiled text (a
    size-independent property; the text itself is sha256-pinned).  At this
    size every tile's look-back spans several 512-tile windows, and tiles
    entered with d > 0 occur."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir, src)
    syn = synth.tiled_stream(hf, text, mib << 20)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(syn.tree)
        # (E.coli at 1 GiB: 4 GiB of output, past 2^31 and 2^32 output bytes)
        out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            out.fill_(0xAB)
            n = dec.decode_device(syn.data, syn.bits, out)
            torch.cuda.synchronize()
            assert n == syn.decoded_bytes
            assert synth.verify_tiled(out, syn)
            assert int(out[n:n + 64].ne(0xAB).sum()) == 0      # nothing written past the end
            assert dec.stats()["exact_fallback"] == 0
    finally:
        dec.close()
        del out
        torch.cuda.empty_cache()


@pytest.mark.parametrize("chunk_kb", [None, 2])
def test_capacity_error_reports_the_total(hh, files_dir, chunk_kb, monkeypatch):
    """A capacity failure returns HH_ERR_CAPACITY with out_len = the
    stream's full symbol count (the size to retry with), the same from
    hh_decode_device and from hh_decode_host, chunk pipeline or not (2 KiB
    chunks: the capacity runs out in an early chunk, the later ones are
    counted only)."""
    import ctypes as C
    import torch
    from huffmandecoderongpus_amd import synth
    if chunk_kb:
        monkeypatch.setenv("HH_PIPE_CHUNK_KB", str(chunk_kb))
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, 1 << 20)
    host = syn.data[: syn.compressed_bytes].cpu().numpy()
    L = hh.lib()
    dec = hh.Decoder(0)
    try:
        dec.set_tree(syn.tree)
        for cap in (syn.decoded_bytes // 3, syn.decoded_bytes - 1):
            buf = np.zeros(cap, np.uint8)
            n = C.c_uint64(0)
            rc = L.hh_decode_host(dec._h, host.ctypes.data, syn.bits, buf.ctypes.data, cap, C.byref(n))
            assert rc == -5 and n.value == syn.decoded_bytes, (rc, n.value)
            d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
            n = C.c_uint64(0)
            rc = L.hh_decode_device(dec._h, syn.data.data_ptr(), syn.bits, d_out.data_ptr(), cap, C.byref(n), None)
            assert rc == -5 and n.value == syn.decoded_bytes, (rc, n.value)
        # and the decoder is usable afterwards
        out = dec.decode_host(host, syn.bits, syn.decoded_bytes)
        assert synth.verify_tiled(torch.from_numpy(out).cuda(), syn)
    finally:
        dec.close()


def test_first_decode_of_fresh_decoders_chunked(hh, files_dir, monkeypatch):
    """The first decode of a new decoder allocates its workspace and zeroes
    its scan ticket; that zeroing must be ordered before the decode's kernels
    on the decoder's (non-blocking) stream.  Round 6's full GPU run caught a
    null-stream hipMemset landing during the first decode's scan: chunked
    hh_decode_host calls on fresh decoders returned 3/16 of the output.  Six
    fresh decoders, each decoding kjv.txt in 512 KiB chunks as its first
    call, every output checked against the reference's text hash."""
    import hashlib
    from huffmandecoderongpus_amd import synth
    monkeypatch.setenv("HH_PIPE_CHUNK_KB", "512")
    hf = hh.HuffFile.load(os.path.join(files_dir, "kjv.txt.huff"))
    for _ in range(6):
        dec = hh.Decoder(0)
        try:
            dec.set_tree(hf.tree())
            out = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
        finally:
            dec.close()
        assert hashlib.sha256(out.tobytes()).hexdigest() == synth.KJV_SHA256


@pytest.mark.parametrize("chunk_kb,mib", [(None, 1024), (4096, 64), (2, 1)])
def test_evaluate_scope_pipeline(hh, files_dir, chunk_kb, mib, monkeypatch):
    """hh_decode_host (the reference's evaluate() scope) uploads the payload
    in chunks, decodes each as a segment entered in the state the previous
    one left and downloads its symbols while later chunks are in flight: the
    bytes must equal the tiled text however many chunks the stream is cut
    into (the default 128 MiB chunks on the 1 GiB stream; 4 MiB chunks; 2 KiB
    chunks, one tile each, on 1 MiB)."""
    import torch
    from huffmandecoderongpus_amd import synth
    if chunk_kb:
        monkeypatch.setenv("HH_PIPE_CHUNK_KB", str(chunk_kb))
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, mib << 20)
    host = syn.data[: syn.compressed_bytes].cpu().numpy()
    dec = hh.Decoder(0)
    try:
        dec.set_tree(syn.tree)
        buf = np.full(syn.decoded_bytes + 64, 0xAB, np.uint8)
        for _ in range(2):
            out = dec.decode_host(host, syn.bits, syn.decoded_bytes + 16, out=buf)
            assert len(out) == syn.decoded_bytes
            assert synth.verify_tiled(torch.from_numpy(out).cuda(), syn)
            assert (buf[syn.decoded_bytes + 16:] == 0xAB).all()
            assert dec.stats()["state_machine"] in (1, 2)
    finally:
        dec.close()


def test_evaluate_scope_keeps_buffers_pinned(hh, files_dir, monkeypatch):
    """HH_FLAG_KEEP_HOST_PINNED: hh_decode_host registers the caller's
    buffers once and reuses the registration -- repeated calls on the same
    buffers, then a NEW output buffer (re-registered), then a longer payload
    view of a new array, then release_host and another call: every output
    equals the tiled text (64 MiB stream, 4 MiB chunks: the pipelined
    path)."""
    import torch
    from huffmandecoderongpus_amd import synth
    monkeypatch.setenv("HH_PIPE_CHUNK_KB", "4096")
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, 64 << 20)
    host = syn.data[: syn.compressed_bytes].cpu().numpy()
    dec = hh.Decoder(0, flags=hh.FLAG_KEEP_HOST_PINNED)
    try:
        dec.set_tree(syn.tree)
        n = syn.decoded_bytes

        def check(out, buf):
            assert len(out) == n
            assert synth.verify_tiled(torch.from_numpy(out).cuda(), syn)
            assert (buf[n + 16:] == 0xAB).all()
        buf = np.full(n + 64, 0xAB, np.uint8)
        for _ in range(3):
            buf[:n] = 0
            check(dec.decode_host(host, syn.bits, n + 16, out=buf), buf)
        buf2 = np.full(n + 64, 0xAB, np.uint8)          # another output buffer
        check(dec.decode_host(host, syn.bits, n + 16, out=buf2), buf2)
        host2 = np.concatenate([host, np.zeros(4096, np.uint8)])   # another payload array
        check(dec.decode_host(host2, syn.bits, n + 16, out=buf2), buf2)
        dec.release_host()
        buf[:n] = 0
        check(dec.decode_host(host, syn.bits, n + 16, out=buf), buf)
        assert dec.stats()["state_machine"] in (1, 2)
    finally:
        dec.close()


def test_kept_pins_follow_the_buffers(hh, files_dir):
    """HH_FLAG_KEEP_HOST_PINNED with buffers that share memory:
    a payload lying inside the output buffer's registration, then a new
    output buffer (the payload must be pinned on its own again), then a
    payload that overlaps the output's registration without being inside it
    -- every call decodes right; and the Python binding refuses the flag
    with a temporary output or a copied payload (freed after the call, their
    address could pass for a registered buffer)."""
    path = os.path.join(files_dir, "paper1.huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    nb, n = (hf.bits + 7) // 8, hf.uncompressedsize
    dec = hh.Decoder(0, flags=hh.FLAG_KEEP_HOST_PINNED)
    try:
        dec.set_tree(hf.tree())
        with pytest.raises(ValueError):
            dec.decode_host(hf.payload, hf.bits, n + 16)                 # (no out)
        with pytest.raises(ValueError):
            dec.decode_host(hf.payload.astype(np.int16), hf.bits, n + 16, out=np.zeros(n + 16, np.uint8))
        X = np.zeros(n + 16 + nb + 4096, np.uint8)
        X[n + 16: n + 16 + nb] = hf.payload
        pay = X[n + 16: n + 16 + nb]                                        # inside out's range
        for _ in range(2):
            got = dec.decode_host(pay, hf.bits, X.size, out=X)
            assert np.array_equal(got, ref)
        Y = np.zeros(n + 64, np.uint8)                                      # the output moves
        for _ in range(2):
            got = dec.decode_host(pay, hf.bits, n + 16, out=Y)
            assert np.array_equal(got, ref)
        Z = np.zeros(n + 16 + nb, np.uint8)                                 # payload at out's tail,
        Z[-nb:] = hf.payload                                                # past the cap given
        got = dec.decode_host(Z[-nb:], hf.bits, n + 16, out=Z)
        assert np.array_equal(got, ref)
        dec.release_host()
        got = dec.decode_host(pay, hf.bits, n + 16, out=Y)
        assert np.array_equal(got, ref)
    finally:
        dec.close()


@pytest.mark.parametrize("env", [{"HH_FRONT_WALK": "2"}, {"HH_FRONT_WALK": "16"},
                                 {"HH_FRONT_WALK": "8192"}, {"HH_EMIT_XPT": "0"},
                                 {"HH_EMIT_XPT": "1"}, {"HH_EMIT_NW": "8"}])
def test_walk_bound_and_deferral_lists(hh, files_dir, env, monkeypatch):
    """Round 2's pipeline (HH_FLAG_LEGACY: k_front -> k_walk -> k_table ->
    k_scan -> k_emit -> k_emitx) moves work out of its waves -- walks longer
    than the front's bound (to k_walk), runs over several regions (to
    k_emitx, through per-wave lists that may fill up) -- and must give the
    same bytes whichever part of it moves: every walk in k_front (8192), a
    few, none (0, the default); no run deferred (0), lists that overflow
    (1); k_emit's 8-wave workgroups.  The knobs are read only by that
    pipeline, so the decoder is built with FLAG_LEGACY and the test asserts
    that pipeline (not the state machine) ran."""
    import torch
    from huffmandecoderongpus_amd import synth
    for k, v in env.items():
        monkeypatch.setenv(k, v)                # read when the tree is set
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, 64 << 20)
    dec = hh.Decoder(0, flags=hh.FLAG_LEGACY)
    try:
        dec.set_tree(syn.tree)
        out = torch.full((syn.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(syn.data, syn.bits, out)
        torch.cuda.synchronize()
        st = dec.stats()
        assert st["state_machine"] == 0 and st["exact_fallback"] == 0 and st["fixed_length"] == 0, st
        assert n == syn.decoded_bytes
        assert synth.verify_tiled(out, syn)
        assert int(out[n:n + 64].ne(0xAB).sum()) == 0
    finally:
        dec.close()


@pytest.mark.parametrize("env", [{"HH_EMF_SWZ": "1"}, {"HH_EMF_SWZ": "0"}, {"HH_EMF_SCO": "0"},
                                 {"HH_EMF_SCO": "0", "HH_EMF_SWZ": "1"}])
def test_emission_staging_variants(hh, files_dir, env, monkeypatch):
    """k_emf's staging and copy-out variants give the same bytes: the
    swizzled staging (chosen for near-uniform codes) forced on kjv's
    variable-length code and off on E.coli's 2-bit code, and the copy-out
    loop instead of the static copy-out (its counted stores) -- each on the
    kjv-tiled and E.coli-tiled streams through the state machine and on
    cut streams of a random tree against the oracle."""
    import torch
    from huffmandecoderongpus_amd import synth
    for k, v in env.items():
        monkeypatch.setenv(k, v)                # read when the tree is set
    monkeypatch.setenv("HH_ONE", "0")           # (k_emf: the two-pass pipeline's emission)
    for src in ("kjv.txt", "E.coli"):
        hf, text = synth.load_source(files_dir, src)
        syn = synth.tiled_stream(hf, text, 16 << 20)
        dec = hh.Decoder(0, flags=hh.FLAG_NO_FIXED)
        try:
            dec.set_tree(syn.tree)
            out = torch.full((syn.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
            n = dec.decode_device(syn.data, syn.bits, out)
            torch.cuda.synchronize()
            st = dec.stats()
            assert st["state_machine"] in (1, 2) and st["exact_fallback"] == 0, (src, st)
            assert n == syn.decoded_bytes, src
            assert synth.verify_tiled(out, syn), src
            assert int(out[n:n + 64].ne(0xAB).sum()) == 0, src
        finally:
            dec.close()
    rng = np.random.default_rng(77)
    iz, io, sy, syms = _random_tree(rng, 40)
    p = rng.dirichlet(np.full(40, 0.5))
    t = hh.Tree(iz, io, sy)
    text = rng.choice(syms, size=300_000, p=p).astype(np.uint8)
    data, bits = t.encode(text)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(t)
        for cut in (bits, bits - 1, bits // 3 + 7):
            ref = _oracle(iz, io, sy, data, cut)
            got = _decode_dev(hh, dec, data, cut, cut + 16)
            assert dec.stats()["state_machine"] in (1, 2)
            assert len(got) == len(ref) and np.array_equal(got, ref), cut
    finally:
        dec.close()


def test_phase_timing_flag(hh, files_dir):
    """HH_FLAG_PHASE_TIMING: events between the count, scan and emission
    kernels give the per-kernel split (ms_sync / ms_scan / ms_emit, summing
    to ms_total); without it only ms_total is measured (the split reads 0).
    The bytes are the same either way."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, 16 << 20)
    outs = []
    for flags in (0, hh.FLAG_PHASE_TIMING):
        dec = hh.Decoder(0, flags=flags)
        try:
            dec.set_tree(syn.tree)
            out = torch.zeros(syn.decoded_bytes + 64, dtype=torch.uint8, device="cuda")
            n = dec.decode_device(syn.data, syn.bits, out)
            torch.cuda.synchronize()
            st = dec.stats()
            assert n == syn.decoded_bytes and st["state_machine"] in (1, 2)
            assert st["ms_total"] > 0
            split = (st["ms_sync"], st["ms_scan"], st["ms_emit"])
            if flags:
                assert all(x > 0 for x in split), st
                assert abs(sum(split) - st["ms_total"]) < 1e-3 * max(1.0, st["ms_total"]), st
            else:
                assert split == (0.0, 0.0, 0.0), st
            outs.append(out)
        finally:
            dec.close()
    assert torch.equal(outs[0], outs[1]) and synth.verify_tiled(outs[0], syn)


@pytest.mark.parametrize("m", ["1", "2", "4"])
def test_count_pass_regions_per_lane(hh, files_dir, m, monkeypatch):
    """The count pass with m consecutive regions per lane (k_cntm: one head
    per lane, the walks read back and rewrite the successor lane's records;
    m = 1: k_cnt, a region per lane) gives the same bytes as the oracle: the kjv- and E.coli-tiled streams
    (the latter through the state machine), cut streams of a 40-leaf and of
    a 256-leaf random tree (7-bit count steps) whose lengths leave partial
    count tiles to the tail launch, and segments entered after a prologue."""
    import torch
    from huffmandecoderongpus_amd import synth
    monkeypatch.setenv("HH_CNT_M", m)           # read when the tree is set
    monkeypatch.setenv("HH_ONE", "0")           # (the two-pass pipeline's count pass)
    for src in ("kjv.txt", "E.coli"):
        hf, text = synth.load_source(files_dir, src)
        syn = synth.tiled_stream(hf, text, 16 << 20)
        dec = hh.Decoder(0, flags=hh.FLAG_NO_FIXED)
        try:
            dec.set_tree(syn.tree)
            out = torch.full((syn.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
            n = dec.decode_device(syn.data, syn.bits, out)
            torch.cuda.synchronize()
            st = dec.stats()
            assert st["state_machine"] in (1, 2) and st["exact_fallback"] == 0, (src, st)
            assert n == syn.decoded_bytes, src
            assert synth.verify_tiled(out, syn), src
            assert int(out[n:n + 64].ne(0xAB).sum()) == 0, src
        finally:
            dec.close()
    rng = np.random.default_rng(91)
    for nleaves, nsym in ((40, 400_000), (256, 300_000)):
        iz, io, sy, syms = _random_tree(rng, nleaves)
        p = rng.dirichlet(np.full(nleaves, 0.5))
        t = hh.Tree(iz, io, sy)
        text = rng.choice(syms, size=nsym, p=p).astype(np.uint8)
        data, bits = t.encode(text)
        dec = hh.Decoder(0)
        try:
            dec.set_tree(t)
            for cut in (bits, bits - 1, bits // 3 + 7, 64 * 256 * 5 + 11):
                if cut > bits:
                    continue
                ref = _oracle(iz, io, sy, data, cut)
                got = _decode_dev(hh, dec, data, cut, cut + 16)
                assert dec.stats()["state_machine"] in (1, 2), nleaves
                assert len(got) == len(ref) and np.array_equal(got, ref), (nleaves, cut)
        finally:
            dec.close()
    # segments: a 4-shard plan of the kjv-tiled stream, each entered after a
    # prologue of 2 tiles, concatenate to the whole
    hf, text = synth.load_source(files_dir, "kjv.txt")
    syn = synth.tiled_stream(hf, text, 4 << 20)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(syn.tree)
        whole = torch.zeros(syn.decoded_bytes + 64, dtype=torch.uint8, device="cuda")
        nw = dec.decode_device(syn.data, syn.bits, whole)
        tb = dec.tile_bits()
        nt = (syn.bits + tb - 1) // tb
        parts, prev_leave = [], 0
        for r in range(4):
            t0, t1 = nt * r // 4, nt * (r + 1) // 4
            pro = min(2, t0)
            b0 = (t0 - pro) * tb
            o = torch.zeros(syn.decoded_bytes + 64, dtype=torch.uint8, device="cuda")
            res = dec.decode_range_ptr(syn.data.data_ptr() + b0 // 8, syn.bits - b0, t1 - t0 + pro, 0,
                                       o.data_ptr(), o.numel(), 0, prologue=pro)
            torch.cuda.synchronize()
            if r:
                assert res["entry_state"] == prev_leave, r
            prev_leave = res["leave_state"]
            parts.append(o[: res["out_len"]])
        cat = torch.cat(parts)
        assert cat.numel() == nw and torch.equal(cat, whole[:nw])
    finally:
        dec.close()


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_legacy_pipeline(hh, files_dir, name):
    """Every fixture through round 2's pipeline (HH_FLAG_LEGACY), device
    side, byte-exact -- the path trees the state machine does not take fall
    back to."""
    import torch
    path = os.path.join(files_dir, name + ".huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec = hh.Decoder(0, flags=hh.FLAG_LEGACY | hh.FLAG_NO_FIXED)
    try:
        dec.set_tree(hf.tree())
        d_in = torch.from_numpy(hf.data.copy()).cuda()
        d_out = torch.zeros(hf.uncompressedsize + 64, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(d_in, hf.bits, d_out)
        torch.cuda.synchronize()
        st = dec.stats()
        assert st["state_machine"] == 0 and st["fixed_length"] == 0 and st["exact_fallback"] == 0, st
        assert n == len(ref)
        assert np.array_equal(d_out[:n].cpu().numpy(), ref)
        assert int(d_out[n:].sum().item()) == 0
    finally:
        dec.close()


def _byte_alphabet_stream(hh, seed, nleaves, nbytes):
    """A natural variable-length code over a byte alphabet: a random tree of
    `nleaves` leaves (nleaves - 1 internal nodes) and i.i.d. symbols from a
    Dirichlet(0.3) distribution over them, encoded by the host encoder to
    about `nbytes` of payload."""
    rng = np.random.default_rng(seed)
    iz, io, sy, syms = _random_tree(rng, nleaves)
    t = hh.Tree(iz, io, sy)
    p = rng.dirichlet(np.full(nleaves, 0.3))
    info = t.info()
    # expected bits per symbol from a sample, to size the text
    probe = rng.choice(syms, size=20000, p=p).astype(np.uint8)
    _, pb = t.encode(probe)
    nsym = int(nbytes * 8 / (pb / probe.size))
    text = rng.choice(syms, size=nsym, p=p).astype(np.uint8)
    data, bits = t.encode(text)
    return iz, io, sy, t, info, text, data, bits


@pytest.mark.parametrize("seed,nleaves", [(11, 256), (12, 256), (13, 200)])
def test_byte_alphabet_code(hh, seed, nleaves):
    """SURVEY 8(a10)'s large trees: a natural variable-length code over 200
    or 256 symbols (199 / 255 internal nodes: more states than round 3's
    state machine took) on a >= 64 MiB stream and on cut streams, through the
    DEFAULT decoder, byte-exact against the oracle's restatement of the
    reference's serial decode (decodeallbits.cl:10-33 accepts any tree)."""
    import torch
    iz, io, sy, t, info, text, data, bits = _byte_alphabet_stream(hh, seed, nleaves, 64 << 20)
    assert info["leaves"] == nleaves and info["reachable"] == 2 * nleaves - 1
    dec = hh.Decoder(0)
    try:
        dec.set_tree(t)
        buf = np.zeros((bits + 7) // 8 + 64, np.uint8)
        buf[: (bits + 7) // 8] = data[: (bits + 7) // 8]
        d_in = torch.from_numpy(buf).cuda()
        d_out = torch.full((text.size + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(d_in, bits, d_out)
        torch.cuda.synchronize()
        st = dec.stats()
        assert st["exact_fallback"] == 0 and st["state_machine"] in (1, 2), st
        assert n == text.size
        assert torch.equal(d_out[:n], torch.from_numpy(text).cuda())
        assert int(d_out[n:n + 64].ne(0xAB).sum()) == 0
        # cut streams (tail rule) against the oracle, on a 4 MiB prefix
        small = min(bits, 32 << 20)
        for cut in (small, small - 1, small // 3 + 7, 1000003):
            ref = _oracle(iz, io, sy, data, cut)
            got = _decode_dev(hh, dec, data, cut, cut + 16)
            assert dec.stats()["exact_fallback"] == 0
            assert len(got) == len(ref) and np.array_equal(got, ref), cut
        # the whole stream against the oracle too (not only the encoder's input)
        ref = _oracle(iz, io, sy, data, bits)
        assert ref.size == text.size and np.array_equal(ref, text)
    finally:
        dec.close()


@pytest.mark.parametrize("mib", [64, 1024])
def test_byte_alphabet_huffman_stream(hh, mib):
    """bench's byte-alphabet workload: a Huffman code over all 256 byte values
    (255 states: 7-bit count steps, 224-bit regions), i.i.d. Zipf bytes
    encoded on the GPU; the default decoder must return the symbols, on the
    state machine; at 64 MiB the payload's first 256 KiB is also checked
    against the host encoder."""
    import torch
    from huffmandecoderongpus_amd import synth
    s = synth.byte_stream(mib << 20)
    if mib == 64:
        pay, _ = s.tree.encode(s.syms[: 1 << 20].cpu().numpy())
        assert np.array_equal(s.data[: 1 << 18].cpu().numpy(), pay[: 1 << 18])
    dec = hh.Decoder(0)
    try:
        dec.set_tree(s.tree)
        assert dec.tile_bits() == 64 * 224
        out = torch.full((s.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            n = dec.decode_device(s.data, s.bits, out)
            torch.cuda.synchronize()
            st = dec.stats()
            assert st["state_machine"] in (1, 2) and st["exact_fallback"] == 0, st
            assert n == s.decoded_bytes
            assert torch.equal(out[:n], s.syms)
            assert int(out[n:n + 64].ne(0xAB).sum()) == 0
    finally:
        dec.close()
        del out, s
        torch.cuda.empty_cache()


@pytest.mark.parametrize("mib", [64, 1024])
def test_iid_stream(hh, files_dir, mib):
    """SURVEY 8d's i.i.d. variant: kjv unigram symbols from splitmix64 (seed
    0x5EED5EED), encoded on the GPU; the decode must return the symbols.  At
    64 MiB the first 1 M symbols are also checked against the host generator
    and the GPU payload's first 256 KiB against the host encoder."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir)
    s = synth.iid_stream(hf, text, mib << 20)
    if mib == 64:
        n0 = 1 << 20
        assert np.array_equal(s.syms[:n0].cpu().numpy(),
                              synth.iid_symbols_np(synth.unigram_cum(text), 0, n0))
        pay, bits = hf.tree().encode(s.syms[:n0].cpu().numpy())
        assert np.array_equal(s.data[: 1 << 18].cpu().numpy(), pay[: 1 << 18])
    dec = hh.Decoder(0)
    try:
        dec.set_tree(s.tree)
        out = torch.full((s.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(s.data, s.bits, out)
        torch.cuda.synchronize()
        assert n == s.decoded_bytes
        assert torch.equal(out[:n], s.syms)
        assert int(out[n:n + 64].ne(0xAB).sum()) == 0
        assert dec.stats()["exact_fallback"] == 0
    finally:
        dec.close()
        del out, s
        torch.cuda.empty_cache()


def test_hufx_over_2gib_save_reload_decode(hh, files_dir, tmp_path):
    """The 64-bit container end to end: a 2.25 GiB kjv-tiled payload (more
    than 2^34 bits, beyond the reference's int32 header) written with
    hh_huff_save, loaded back with hh_huff_load and decoded on the GPU."""
    import torch
    from huffmandecoderongpus_amd import synth
    hf, text = synth.load_source(files_dir)
    syn = synth.tiled_stream(hf, text, (9 << 30) // 4)
    assert syn.bits > 1 << 34
    nb = syn.compressed_bytes
    data = np.zeros(nb + hh.PAYLOAD_PAD, np.uint8)
    data[:nb] = syn.data[:nb].cpu().numpy()
    big = hh.HuffFile(syn.tree.izero, syn.tree.ione, syn.tree.sym, syn.bits, syn.decoded_bytes, data)
    path = str(tmp_path / "kjv_2g.huff")
    big.save(path)
    del big
    back = hh.HuffFile.load(path)
    assert back.bits == syn.bits and back.uncompressedsize == syn.decoded_bytes
    dec = hh.Decoder(0)
    try:
        dec.set_tree(back.tree())
        d_in = torch.from_numpy(back.data).cuda()
        del back
        out = torch.empty(syn.decoded_bytes + 4096, dtype=torch.uint8, device="cuda")
        n = dec.decode_device(d_in, syn.bits, out)
        torch.cuda.synchronize()
        assert n == syn.decoded_bytes
        assert synth.verify_tiled(out, syn)
    finally:
        dec.close()
        os.remove(path)
        torch.cuda.empty_cache()


@pytest.mark.parametrize("name,world,probe", [("kjv.txt", 3, 2), ("kjv.txt", 5, 1), ("kjv.txt", 4, 0),
                                               ("hello", 4, 2), ("paper1", 40, 2)])
def test_segments_concatenate(hh, files_dir, name, world, probe):
    """hh_decode_device_range on one GPU, shards planned as bench.py --gpus N
    plans them, each with `probe` predecessor tiles as a prologue; every
    "rank" is a thread running shard.settle over an in-process gather (one
    decoder, calls serialised).  probe 0: entries are guesses that the
    exchange must catch.  hello (1 tile) and paper1 (< 40 tiles): more ranks
    than tiles, the empty shards pass ntiles 0.  The outputs must
    concatenate to the oracle's."""
    import torch
    from huffmandecoderongpus_amd import shard
    path = os.path.join(files_dir, name + ".huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec = hh.Decoder(0)
    try:
        dec.set_tree(hf.tree())
        tb = dec.tile_bits()
        pay = torch.zeros(len(hf.payload) + 256, dtype=torch.uint8, device="cuda")
        pay[:len(hf.payload)] = torch.from_numpy(hf.payload.copy()).cuda()
        segs = [shard.plan(hf.bits, tb, world, r, probe) for r in range(world)]
        outs = [torch.zeros(hf.bits + 64, dtype=torch.uint8, device="cuda") for _ in segs]
        final, redone = _settle_segments(dec, pay, segs, outs)
        got = torch.cat([outs[r][:final[r]["out_len"]] for r in range(world)]).cpu().numpy()
        assert len(got) == len(ref) and np.array_equal(got, ref)
        ntiles = (hf.bits + tb - 1) // tb
        if probe:
            # (a rank without a tile of its own takes its predecessor's leave
            # state in one exchange round: only those are redone)
            assert sum(n for n, s in zip(redone, segs) if s.t1 > s.t0) == 0
        elif ntiles >= world:
            assert sum(redone) >= 1
    finally:
        dec.close()


def _settle_segments(dec, pay, segs, outs):
    """Every segment decoded with hh_decode_device_range on this one GPU, one
    thread per "rank" running shard.settle over an in-process gather (calls
    serialised on one decoder).  Returns (final results, redo counts)."""
    import threading
    import torch
    from huffmandecoderongpus_amd import shard
    world = len(segs)
    tb = segs[0].tile_bits
    lock = threading.Lock()
    bar = threading.Barrier(world)
    slots = [None] * world
    final = [None] * world
    redone = [0] * world
    errors = []

    def run(r, in_state, prologue):
        s = segs[r]
        skip = s.prologue - prologue
        with lock:
            # (a shard with no tile of its own: ntiles 0 through the C ABI)
            res = dec.decode_range_ptr(pay.data_ptr() + (s.buf_bit + skip * tb) // 8,
                                       s.bits_avail - skip * tb,
                                       s.ntiles - skip if s.t1 > s.t0 else 0, in_state,
                                       outs[r].data_ptr(), outs[r].numel(), 0,
                                       prologue=prologue)
            torch.cuda.synchronize()
        res["in_state"] = res["entry_state"]
        return res

    def rank_main(r):
        try:
            def gather(vals):
                slots[r] = list(vals)
                bar.wait()
                rows = [list(x) for x in slots]
                bar.wait()
                return rows

            def redo(st):
                redone[r] += 1
                return run(r, st, 0)

            first = run(r, 0, segs[r].prologue)
            if segs[r].prologue == 0 and segs[r].t0 > 0:
                first["entry_exact"] = False
            final[r] = shard.settle(first, redo, gather, r, world)[0]
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors
    return final, redone


def test_eight_shards_of_the_8gib_stream():
    """BASELINE.json configs[3] on one GPU: the 8 GiB kjv-tiled stream cut
    into the 8 shards bench.py --gpus 8 plans (1 GiB each, 2 prologue
    tiles), every shard decoded with hh_decode_device_range, entry states
    settled; each shard's output must equal the tiled text from its base and
    the bases must add up to the whole stream's symbol count."""
    import torch
    from huffmandecoderongpus_amd import shard, synth
    H = pytest.importorskip("huffmandecoderongpus_amd")
    hf, text = synth.load_source(os.path.join(ROOT, "files"))
    world = 8
    syn = synth.tiled_stream(hf, text, world << 30)
    dec = H.Decoder(0)
    try:
        dec.set_tree(syn.tree)
        tb = dec.tile_bits()
        segs = [shard.plan(syn.bits, tb, world, r) for r in range(world)]
        minlen = int(min(v for v in synth.code_lengths(syn.tree) if v > 0))
        outs = [torch.empty(s.owned_bits // minlen + 4096, dtype=torch.uint8, device="cuda")
                for s in segs]
        final, redone = _settle_segments(dec, syn.data, segs, outs)
        assert sum(redone) == 0                       # every prologue was exact
        L = syn.text.numel()
        base = 0
        for r in range(world):
            n = final[r]["out_len"]
            for o in range(0, n, 1 << 28):
                m = min(1 << 28, n - o)
                idx = (torch.arange(m, device="cuda", dtype=torch.int64) + (base + o)) % L
                assert torch.equal(outs[r][o:o + m], syn.text[idx]), (r, o)
            base += n
        assert base == syn.decoded_bytes
    finally:
        dec.close()
        del outs
        torch.cuda.empty_cache()


def _shard_rank(rank, world, port, mib, q, backend="gloo", probe=2):
    import torch
    import torch.distributed as dist
    import huffmandecoderongpus_amd as H
    from huffmandecoderongpus_amd import shard, synth
    try:
        if backend == "nccl":
            torch.cuda.set_device(0)
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}",
                                rank=rank, world_size=world)
        torch.cuda.set_device(0)
        hf, text = synth.load_source(os.path.join(ROOT, "files"))
        job = shard.ShardJob(hf, text, mib << 20, rank, world, 0, probe=probe, wrong_entry=probe == 0)
        job.check_step()                     # the checked step: decode + exchange
        torch.cuda.synchronize()
        ok = job.verify()
        job.out.fill_(0)
        for _ in range(3):                   # timed steps: decodes only, queued
            job.decode_step()
        job.wait()
        torch.cuda.synchronize()
        ok = ok and job.verify()             # (the timed steps' output)
        ok = ok and job.confirm()            # the exchange after them agrees
        job.out.fill_(0)
        ok = ok and job.pipelined_steps(3)   # bench's timed steps: decode, exchange, redo, pipelined
        torch.cuda.synchronize()
        ok = ok and job.verify()             # (the last pipelined step's output)
        rep = job.gather_report()            # the assembled stream (gloo: host tensors)
        ok = ok and rep["allgather"]["seams_ok"]
        q.put((rank, ok, job.decoded_bytes, job.seg.prologue, job.redo_state))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), 0, 0, None))


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("probe", [2, 0])
def test_shard_job_two_ranks_one_gpu(probe):
    """bench.py's multi-GPU path (ShardJob: shard plan, prologue entry, the
    checked step's settle exchange, decode-only steps queued asynchronously
    with no collective, the exchange after them confirming the checked rows,
    the pipelined full steps (each with its own exchange and redo),
    per-rank verification against the tiled text, the all-gather assembly
    checked on rank 0) with two processes sharing GPU 0 over gloo (RCCL
    needs distinct GPUs).  probe 0: rank 1 has no prologue and enters in a
    state known to be wrong (ShardJob wrong_entry): the checked step's
    exchange must catch it and the timed steps must include its redo."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_shard_rank, args=(r, 2, port, 32, q, "gloo", probe)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted((q.get(timeout=300) for _ in ps), key=lambda g: g[0])
    for p in ps:
        p.join(timeout=60)
    for rank, ok, n, pro, redo in got:
        assert ok is True, (rank, ok)
        assert n > 0
    if probe:
        assert got[1][3] > 0 and got[1][4] is None    # rank 1 decoded a prologue, entry right
    else:
        assert got[1][3] == 0 and got[1][4] is not None   # guessed entry wrong: redone


def test_shard_job_over_rccl_one_rank():
    """The same ShardJob path over RCCL (backend "nccl"), one rank on GPU 0:
    the settle exchange and the output all-gather run as RCCL collectives on
    device tensors (all_gather, all_gather_into_tensor) -- the code the
    multi-GPU bench runs on N GPUs (RCCL refuses two ranks on one GPU)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_shard_rank, args=(0, 1, port, 32, q, "nccl"))
    p.start()
    rank, ok, n, pro, redo = q.get(timeout=300)
    p.join(timeout=60)
    assert ok is True, ok
    assert n > 0 and pro == 0


@pytest.mark.parametrize("name", ["hello", "paper1", "news", "kjv.txt", "E.coli"])
def test_segment_path_fixtures(hh, files_dir, name):
    """The segment path (HH_FLAG_FORCE_SEGMENT), byte-exact on the fixtures."""
    path = os.path.join(files_dir, name + ".huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    dec = hh.Decoder(0, flags=2)
    try:
        dec.set_tree(hf.tree())
        out = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
        assert dec.stats()["exact_fallback"] == 2
        assert np.array_equal(out, ref)
    finally:
        dec.close()


def test_async_decodes(hh, files_dir):
    """hh_decode_device_async / hh_decode_wait: decodes of different streams
    enqueued back to back, each checked while the next runs (alternating
    result slots) -- the state machine (kjv), k_fixed (E.coli), a random tree's
    cut stream, and the same decoder reused -- every output and length
    byte-exact against the oracle after the wait; a capacity failure among
    them is reported by the wait (the others still decode), and synchronous
    calls after asynchronous ones see a drained decoder."""
    import torch
    jobs = []
    for name in ("kjv.txt", "E.coli", "paper1"):
        path = os.path.join(files_dir, name + ".huff")
        hf = hh.HuffFile.load(path)
        jobs.append((hf.tree(), hf.data, hf.bits, O.OracleHuff.load(path).chain_decode()))
    rng = np.random.default_rng(31)
    iz, io, sy, syms = _random_tree(rng, 60)
    t = hh.Tree(iz, io, sy)
    data, bits = t.encode(rng.choice(syms, size=400_000, p=rng.dirichlet(np.full(60, 0.4))).astype(np.uint8))
    for cut in (bits, bits // 2 + 3):
        jobs.append((t, data, cut, _oracle(iz, io, sy, data, cut)))
    decs = {}
    try:
        for rep in range(2):
            pend = []
            for k, (tree, data, bits, ref) in enumerate(jobs):
                dec = decs.get(k % 3)
                if dec is None:
                    dec = decs[k % 3] = hh.Decoder(0)
                dec.set_tree(tree)
                buf = np.zeros(((bits + 7) // 8 + 64 + 3) // 4 * 4, np.uint8)
                buf[: (bits + 7) // 8] = np.asarray(data, np.uint8)[: (bits + 7) // 8]
                d_in = torch.from_numpy(buf).cuda()
                d_out = torch.full((len(ref) + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
                # the same decoder twice in a row: two decodes in flight on it
                for _ in range(2):
                    n = dec.decode_device_async(d_in, bits, d_out)
                    pend.append((dec, n, d_out, ref))
                dec.wait() if rep == 1 else None
            for dec in decs.values():
                dec.wait()
            for dec, n, d_out, ref in pend:
                assert n.value == len(ref)
                got = d_out[: n.value].cpu().numpy()
                assert np.array_equal(got, ref)
                assert int(d_out[n.value: n.value + 64].ne(0xAB).sum()) == 0
        # a capacity failure is the wait's; the decode after it is fine
        tree, data, bits, ref = jobs[0]
        dec = decs[0]
        dec.set_tree(tree)
        buf = np.zeros(((bits + 7) // 8 + 64 + 3) // 4 * 4, np.uint8)
        buf[: (bits + 7) // 8] = np.asarray(data, np.uint8)[: (bits + 7) // 8]
        d_in = torch.from_numpy(buf).cuda()
        small = torch.zeros(len(ref) // 2, dtype=torch.uint8, device="cuda")
        d_out = torch.zeros(len(ref) + 64, dtype=torch.uint8, device="cuda")
        dec.decode_device_async(d_in, bits, small)
        n = dec.decode_device_async(d_in, bits, d_out)
        with pytest.raises(hh.HipHuffError):
            dec.wait()
        assert n.value == len(ref) and np.array_equal(d_out[: n.value].cpu().numpy(), ref)
        dec.wait()                                      # (cleared)
        # a synchronous decode right after an asynchronous one
        dec.decode_device_async(d_in, bits, d_out)
        assert dec.decode_device(d_in, bits, d_out) == len(ref)
        dec.wait()
    finally:
        for dec in decs.values():
            dec.close()


def test_async_decodes_on_two_streams(hh, files_dir):
    """Asynchronous decodes alternating between two torch streams on ONE
    decoder (its workspace is shared): each decode must wait for the pending
    one's emission before its count pass rewrites the records -- kjv.txt and
    a 64 MiB tiled stream, alternately, eight decodes, every output and
    length checked after the wait."""
    import torch
    from huffmandecoderongpus_amd import synth
    path = os.path.join(files_dir, "kjv.txt.huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    text = torch.from_numpy(ref.copy()).cuda()
    syn = synth.tiled_stream(hf, ref, 64 << 20, device=torch.device("cuda", 0))
    buf = np.zeros(((hf.bits + 7) // 8 + 64 + 3) // 4 * 4, np.uint8)
    buf[: (hf.bits + 7) // 8] = hf.data[: (hf.bits + 7) // 8]
    small_in = torch.from_numpy(buf).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dec = hh.Decoder(0)
    try:
        dec.set_tree(hf.tree())
        outs = [torch.full(((syn.decoded_bytes if k % 2 == 0 else len(ref)) + 4096,), 0xAB,
                           dtype=torch.uint8, device="cuda") for k in range(8)]
        torch.cuda.synchronize()          # (inputs and outputs made on the default stream)
        pend = []
        for k, out in enumerate(outs):
            s = streams[k % 2]
            if k % 2 == 0:
                pend.append(("big", dec.decode_device_async(syn.data, syn.bits, out, s), out))
            else:
                pend.append(("small", dec.decode_device_async(small_in, hf.bits, out, s), out))
        dec.wait()
        torch.cuda.synchronize()
        for kind, n, out in pend:
            if kind == "big":
                assert n.value == syn.decoded_bytes and synth.verify_tiled(out, syn)
            else:
                assert n.value == len(ref) and torch.equal(out[: n.value], text)
            assert int(out[n.value: n.value + 64].ne(0xAB).sum()) == 0
        assert dec.stats()["state_machine"] in (1, 2)
    finally:
        dec.close()
        del syn
        torch.cuda.empty_cache()


def test_async_decode_exact_fallback(hh, files_dir, monkeypatch):
    """The asynchronous path's exact fallback (async_check): a decode whose
    chains are reported not to meet (HH_TEST_NOSYNC=1, the test hook that
    makes every state-machine decode report it) is found failed while the
    NEXT decode is already queued, and is decoded again on the segment path
    through its saved arguments (output pointer, capacity, out_len pointer).
    Three decodes of kjv.txt queued back to back into three buffers, then the
    wait: every output and length equals the oracle's, and the fallback is
    the segment path."""
    import torch
    monkeypatch.setenv("HH_TEST_NOSYNC", "1")
    path = os.path.join(files_dir, "kjv.txt.huff")
    hf = hh.HuffFile.load(path)
    ref = O.OracleHuff.load(path).chain_decode()
    buf = np.zeros(((hf.bits + 7) // 8 + 64 + 3) // 4 * 4, np.uint8)
    buf[: (hf.bits + 7) // 8] = hf.data[: (hf.bits + 7) // 8]
    d_in = torch.from_numpy(buf).cuda()
    dec = hh.Decoder(0)
    try:
        dec.set_tree(hf.tree())
        outs = [torch.full((len(ref) + 4096,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(3)]
        ns = [dec.decode_device_async(d_in, hf.bits, o) for o in outs]
        dec.wait()
        torch.cuda.synchronize()
        st = dec.stats()
        assert st["exact_fallback"] == 2 and st["repairs"] == 1
        for n, o in zip(ns, outs):
            assert n.value == len(ref)
            assert np.array_equal(o[: n.value].cpu().numpy(), ref)
            assert int(o[n.value: n.value + 64].ne(0xAB).sum()) == 0
    finally:
        dec.close()


def test_non_resynchronising_code_takes_the_segment_path(hh):
    """An 11-bit fixed-length code with 96-bit regions realigns only every 11
    regions (> HH_KM): the walks fail and the decoder must switch to the
    exact O(N) segment path, not mis-decode."""
    iz, io, sy = _complete_tree(11)
    rng = np.random.default_rng(11)
    bits = 11 * 300000 + 5
    data = rng.integers(0, 256, size=bits // 8 + 1).astype(np.uint8)
    ref = _oracle(iz, io, sy, data, bits)
    dec = hh.Decoder(0, lane_bits=96)
    try:
        dec.set_tree(hh.Tree(iz, io, sy))
        got = _decode_dev(hh, dec, data, bits, bits)
        assert dec.stats()["exact_fallback"] == 2
        assert len(got) == len(ref) and np.array_equal(got, ref)
    finally:
        dec.close()


def test_non_resynchronising_code_beyond_2_31_bits(hh):
    """The same code on a 2.2e9-bit stream (past the stage pipeline's int32
    cap): 200 M random symbols encoded on the GPU, decoded by the segment
    path, compared with the symbols."""
    import torch
    from huffmandecoderongpus_amd import synth
    iz, io, sy = _complete_tree(11)
    tree = hh.Tree(iz, io, sy)
    code, lens = synth.code_table(tree)
    n = 200_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    payload, bits = synth.encode_gpu(syms, code, lens)
    assert bits == 11 * n and bits > 1 << 31
    dec = hh.Decoder(0, lane_bits=96)
    try:
        dec.set_tree(tree)
        out = torch.full((n + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
        got = dec.decode_device(payload, bits, out)
        torch.cuda.synchronize()
        assert dec.stats()["exact_fallback"] == 2
        assert got == n
        assert torch.equal(out[:n], syms)
        assert int(out[n:n + 64].ne(0xAB).sum()) == 0
    finally:
        dec.close()
        del out, payload, syms
        torch.cuda.empty_cache()


@pytest.mark.parametrize("name,mib", [("E.coli", 0), ("E.coli", 1024)])
def test_state_machine_on_a_fixed_length_code(hh, files_dir, name, mib):
    """BASELINE config 5's general path: E.coli's 2-bit code with k_fixed
    off (HH_FLAG_NO_FIXED) goes through the state machine (every region's
    guess is right, the densest output: 4 symbols per byte).  The fixture
    against the oracle; the 1 GiB tiled stream (4 GiB of output) against the
    tiled text."""
    import torch
    from huffmandecoderongpus_amd import synth
    dec = hh.Decoder(0, flags=hh.FLAG_NO_FIXED)
    try:
        if mib == 0:
            path = os.path.join(files_dir, name + ".huff")
            hf = hh.HuffFile.load(path)
            ref = O.OracleHuff.load(path).chain_decode()
            dec.set_tree(hf.tree())
            out = dec.decode_host(hf.payload, hf.bits, hf.uncompressedsize + 3)
            st = dec.stats()
            assert st["state_machine"] in (1, 2) and st["fixed_length"] == 0
            assert np.array_equal(out, ref)
        else:
            hf, text = synth.load_source(files_dir, name)
            syn = synth.tiled_stream(hf, text, mib << 20)
            dec.set_tree(syn.tree)
            out = torch.full((syn.decoded_bytes + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
            n = dec.decode_device(syn.data, syn.bits, out)
            torch.cuda.synchronize()
            st = dec.stats()
            assert st["state_machine"] in (1, 2) and st["fixed_length"] == 0
            assert n == syn.decoded_bytes and synth.verify_tiled(out, syn)
            assert int(out[n:n + 64].ne(0xAB).sum()) == 0
            del out, syn
            torch.cuda.empty_cache()
    finally:
        dec.close()


def _caterpillar(depth):
    """Symbol k < depth: k ones then a zero (k + 1 bits); symbol depth:
    depth ones.  Internal node k holds symbol k as its tail-rule byte."""
    # node 2k: internal, its zero child 2k+1 a leaf, its one child 2k+2
    n = 2 * depth + 1
    izero = np.full(n, -1, np.int32)
    ione = np.full(n, -1, np.int32)
    sym = np.zeros(n, np.uint8)
    for k in range(depth):
        izero[2 * k], ione[2 * k], sym[2 * k] = 2 * k + 1, 2 * k + 2, k
        sym[2 * k + 1] = k
    sym[2 * depth] = depth
    return izero, ione, sym


def test_long_codes_beyond_2_31_bits(hh):
    """Codes of up to 40 bits (a caterpillar tree: 40 states) through the
    state machine on a stream of more than 2^31 bits: 110 M symbols drawn
    uniformly (20.5 bits on average), encoded on the GPU, decoded, compared
    with the symbols.  Round 2 sent codes over 32 bits to the O(bits log)
    stage pipeline, capped below 2^31 bits."""
    import torch
    from huffmandecoderongpus_amd import synth
    iz, io, sy = _caterpillar(40)
    tree = hh.Tree(iz, io, sy)
    code, lens = synth.code_table(tree, max_len=40)
    assert lens.max() == 40
    n = 110_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(40)
    syms = torch.randint(0, 41, (n,), dtype=torch.uint8, device="cuda", generator=g)
    payload, bits = synth.encode_gpu(syms, code, lens)
    assert bits > 1 << 31
    dec = hh.Decoder(0)
    try:
        dec.set_tree(tree)
        out = torch.full((n + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
        got = dec.decode_device(payload, bits, out)
        torch.cuda.synchronize()
        st = dec.stats()
        assert st["state_machine"] in (1, 2) and st["exact_fallback"] == 0
        assert got == n
        assert torch.equal(out[:n], syms)
        assert int(out[n:n + 64].ne(0xAB).sum()) == 0
    finally:
        dec.close()
        del out, payload, syms
        torch.cuda.empty_cache()


def test_copy_probe(hh):
    """hh_copy_device (bench.py's streaming-copy reference): both cache
    policies copy every byte (an odd number of 16-B elements, not a multiple
    of the kernel's stride), and a misaligned size is an argument error."""
    import torch
    n = (1 << 24) + 16 * 37
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    for nt in (False, True):
        b = torch.zeros_like(a)
        ms = hh.copy_device(a, b, nt)
        torch.cuda.synchronize()
        assert ms > 0 and torch.equal(a, b)
    with pytest.raises(hh.HipHuffError):
        hh.copy_device(a[:17], torch.zeros(17, dtype=torch.uint8, device="cuda"))


@pytest.mark.parametrize("nleaves,seed", [(300, 41), (500, 42)])
def test_tree_beyond_the_state_machine_default_path(hh, nleaves, seed):
    """A tree of more than 256 leaves (symbols repeat: the reference's loader
    takes any node count, huffdata.c:41-54, and decodeallbits.cl:10-33 walks
    any tree) has more than 255 internal nodes, past the state machine: the
    DEFAULT decoder must still be exact -- random payload bits (every bit
    string decodes with a complete tree) cut at several points, against the
    oracle, through hh_decode_device and the evaluate() scope."""
    rng = np.random.default_rng(seed)
    izl, iol, leaves = [-1], [-1], [0]
    while len(leaves) < nleaves:                    # random splits of random leaves
        v = leaves.pop(int(rng.integers(len(leaves))))
        a = len(izl)
        izl[v], iol[v] = a, a + 1
        izl += [-1, -1]
        iol += [-1, -1]
        leaves += [a, a + 1]
    iz, io = np.array(izl), np.array(iol)
    sy = rng.integers(0, 256, size=len(iz)).astype(np.uint8)     # repeated symbols
    sy[iz != -1] = 0
    t = hh.Tree(iz, io, sy)
    info = t.info()
    assert info["leaves"] == nleaves and nleaves - 1 > 255
    nbytes = 400_000
    data = rng.integers(0, 256, size=nbytes).astype(np.uint8)
    dec = hh.Decoder(0)
    try:
        dec.set_tree(t)
        for cut in (nbytes * 8, nbytes * 8 - 5, 123_457):
            ref = _oracle(iz, io, sy, data, cut)
            got = _decode_dev(hh, dec, data, cut, cut + 16)
            st = dec.stats()
            assert st["state_machine"] == 0
            assert len(got) == len(ref) and np.array_equal(got, ref), (cut, st)
        pay = np.zeros(nbytes + 64, np.uint8)
        pay[:nbytes] = data
        out = dec.decode_host(pay[:nbytes], nbytes * 8, nbytes * 8 + 16)
        assert np.array_equal(out, _oracle(iz, io, sy, data, nbytes * 8))
    finally:
        dec.close()
