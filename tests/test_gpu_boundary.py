"""The drop-in boundary on the GPU: the reference's own harness driving the
HIP plugin, the HuffFramework CLI, and the reference-shaped stage kernels'
intermediate arrays against the golden hello trace and the oracle's pes
restatement (framework/pes.c:22-104)."""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = os.path.join(ROOT, "files")
CLI = os.path.join(ROOT, "build", "HuffFramework")
LINE = r"^\s*{dec}\s+{name}\s+\d+\.\d{{9}} ms$"

ALL = ["hello", "paper1", "news", "book2", "bible.txt", "world192.txt", "kjv.txt", "E.coli"]


@pytest.mark.gpu
@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref/libhuffref.so not built")
def test_reference_harness_evaluates_hip_plugin():
    """newDecoder(hipHuffApproach, NULL, "hip") + the reference's evalandshow
    -> evaluate -> compareUnCompressedData on every fixture (a mismatch is
    err(1, "decode problem") inside the reference code: exit status 1)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "harness_ref.py")] + ALL,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    for name in ALL:
        pat = re.compile(LINE.format(dec="hip", name=re.escape(name)))
        assert any(pat.match(ln) for ln in lines), (name, lines)
    assert "different" not in r.stdout


@pytest.fixture(scope="module")
def full_files(tmp_path_factory):
    """files/ plus the regenerated kjv.txt and E.coli originals (sha256-checked,
    tools/regen_files.py), so the CLI byte-compares every decode."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import regen_files
    return regen_files.regen(str(tmp_path_factory.mktemp("files_full")))


@pytest.mark.gpu
@pytest.mark.parametrize("test,name", [("hello", "hello"), ("kjvprof", "kjv")])
def test_cli_prints_the_reference_line(test, name, full_files):
    if not os.path.exists(CLI):
        pytest.skip("build/HuffFramework not built")
    env = dict(os.environ, HIPHUFF_FILES=full_files)
    r = subprocess.run([CLI, test, "--reps", "3"], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "absent" not in r.stderr                   # byte-compared, not length-checked
    assert re.search(LINE.format(dec="hip", name=name), r.stdout, re.M), r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("test,n_min", [("quickgraph2", 20), ("graph2", 40)])
def test_cli_graphtest_byte_checked(test, n_min, full_files):
    """graphtest (framework/mainrun.c:387-410): every prefix cut at a symbol
    boundary (setTargetSizes, mainrun.c:361-385) is decoded and byte-compared
    with the original's prefix (exit status 1 on a mismatch); kjv.txt is the
    regenerated original, so graph2 is checked byte for byte too."""
    if not os.path.exists(CLI):
        pytest.skip("build/HuffFramework not built")
    r = subprocess.run([CLI, test, "--files", full_files, "--reps", "1"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "absent" not in r.stderr
    rows = [ln.split() for ln in r.stdout.splitlines() if re.match(r"^\s*\d+\s+\d+\.\d{9}$", ln)]
    assert len(rows) >= n_min, r.stdout[-2000:]
    sizes = [int(x[0]) for x in rows]
    assert sizes == sorted(sizes) and len(set(sizes)) == len(sizes)


def _jacobi_calcbitsindex(levels, bits, nsteps):
    """calcbitsindex.cl:5-22 with every read taken before every write of a
    step (the synchronous reading of the parallel kernel)."""
    idx = np.full(bits, -1, np.int64)
    idx[0] = 0
    after = {}
    pw = 1 << (nsteps - 1)
    for step in range(nsteps, 0, -1):
        off = levels[step - 1].astype(np.int64)
        b = np.nonzero((off != -1) & (idx != -1))[0]
        tgt = b + off[b]
        keep = tgt < bits
        new = idx.copy()
        new[tgt[keep]] = idx[b[keep]] + pw
        idx = new
        after[step] = idx.copy()
        pw >>= 1
    return after


def _stage_case(name):
    import torch
    import huffmandecoderongpus_amd as H
    hf = H.HuffFile.load(os.path.join(FILES, name + ".huff"))
    pes = O.OracleHuff.load(os.path.join(FILES, name + ".huff")).pes()
    B = hf.bits
    dec = H.Decoder(0)
    L = H.lib()
    try:
        dec.set_tree(hf.tree())
        d_in = torch.from_numpy(hf.data.copy()).cuda()
        idx = torch.zeros(B, dtype=torch.int32, device="cuda")
        bitdecode = torch.zeros(B, dtype=torch.uint8, device="cuda")
        steps = torch.full((25, B), 12345, dtype=torch.int32, device="cuda")
        result = torch.zeros(B, dtype=torch.uint8, device="cuda")
        s = 0   # default stream (ordered with torch's work)
        got = {}
        assert L.hh_stage_initbitsindex(dec._h, idx.data_ptr(), B, s) == 0
        torch.cuda.synchronize()
        got["init"] = idx.cpu().numpy().copy()
        assert L.hh_stage_decodeallbits(dec._h, d_in.data_ptr(), B, bitdecode.data_ptr(),
                                        steps.data_ptr(), s) == 0
        flags = []
        step = 0
        import ctypes as C
        while True:
            fl = C.c_int32(0)
            assert L.hh_stage_makebigtable(dec._h, B, steps.data_ptr(), step, C.byref(fl), s) == 0
            flags.append(fl.value)
            step += 1
            if fl.value == -1:
                break
        torch.cuda.synchronize()
        got["bitdecode"] = bitdecode.cpu().numpy()
        got["levels"] = steps[: step + 1].cpu().numpy()
        got["flags"] = flags
        zero = torch.zeros(1, dtype=torch.int32, device="cuda")
        idx[0:1].copy_(zero)
        pw = 1 << (step - 1)
        got["idx_after"] = {}
        for k in range(step, 0, -1):
            assert L.hh_stage_calcbitsindex(dec._h, B, idx.data_ptr(), steps.data_ptr(), k, pw, s) == 0
            torch.cuda.synchronize()
            got["idx_after"][k] = idx.cpu().numpy().copy()
            pw >>= 1
        assert L.hh_stage_calcresult(dec._h, B, idx.data_ptr(), bitdecode.data_ptr(),
                                     result.data_ptr(), s) == 0
        mx = C.c_int32(0)
        assert L.hh_stage_findmax(dec._h, B, idx.data_ptr(), C.byref(mx), s) == 0
        torch.cuda.synchronize()
        got["maxvalue"] = mx.value
        got["result"] = result[: mx.value + 1].cpu().numpy()
        return hf, pes, got, step
    finally:
        dec.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hello", "paper1"])
def test_stage_kernels_intermediate_arrays(name):
    """Every intermediate array of the six reference-shaped kernels
    (k_st_*) against the oracle's pes restatement (pes.c:22-104), and for
    hello against the golden trace."""
    hf, pes, got, nsteps = _stage_case(name)
    B = hf.bits
    assert (got["init"] == -1).all()                                   # initbitsindex
    assert np.array_equal(got["bitdecode"], pes["bitdecode"])          # decodeallbits
    assert nsteps == pes["nlevels"]
    assert np.array_equal(got["levels"], pes["steps"])                 # every makebigtable level
    assert got["flags"] == [int(v) for v in pes["steps"][:nsteps, 0]]  # the 4-byte flag reads
    # calcbitsindex: every step's array holds at least the synchronous
    # (Jacobi) step's entries, and every entry it holds is the final index
    # of that bit (the reference's benign same-launch read)
    jac = _jacobi_calcbitsindex(got["levels"], B, nsteps)
    final = pes["bitsindex"]
    for k, arr in got["idx_after"].items():
        set_g = arr != -1
        assert (set_g >= (jac[k] != -1)).all(), k
        assert np.array_equal(arr[set_g], final[set_g]), k
    assert np.array_equal(got["idx_after"][1], final)                 # after the last step
    assert np.array_equal(got["result"], pes["result"])               # calcresult
    assert got["maxvalue"] + 1 == hf.uncompressedsize                 # findmax
    if name == "hello":
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "hello_pes.json")))
        assert g["nlevels"] == nsteps
        assert [list(r) for r in got["levels"]] == g["levels"]
        assert list(got["bitdecode"]) == g["bitdecode"]
        assert list(got["idx_after"][1]) == g["bitsindex"]
        assert bytes(got["result"]).decode() == g["result"] == "Hello World"
