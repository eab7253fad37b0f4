"""Run the REFERENCE's own harness on the HIP plugin (test helper, GPU only).

    python tests/harness_ref.py NAME [NAME ...]

For each fixture NAME (files/NAME + files/NAME.huff) this loads the data with
the reference's own loadTestData (framework/huffdata.c:205-215, compiled into
oracle/_ref/libhuffref.so by oracle/Makefile), registers hipHuffApproach
(libhiphuff.so) with the reference's newDecoder (framework/decodeUtil.c:16-24)
exactly as mainrun.c:480-488 registers its GPU decoders, and calls the
reference's evalandshow -> evaluate (framework/mainrun.c:412-420,
decodeUtil.c:30-70): one decode checked by compareUnCompressedData
(huffdata.c:183-203; a mismatch ends the process with err(1, "decode
problem")), then REPEATS timed decodes.  It prints the reference's own
"%17s %8s     %.9f ms" line per fixture.

kjv.txt and E.coli are absent from the reference tree (.MISSING_LARGE_BLOBS);
their originals are regenerated here by the oracle's serial decoder and
checked against the sha256 digests recorded in BASELINE.md before use.
"""
import ctypes as C
import hashlib
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DIGESTS = {   # BASELINE.md / SURVEY.md 8(c)
    "kjv.txt": "e4e21579f6360b35e66dc97b67cd732a3f759623e41e4e077bec039eeb79fd0a",
    "E.coli": "9125dfd87315961ef4286f3856098069e050cc3a2abe65735fe43e69d1996f40",
}


def main(names):
    import huffmandecoderongpus_amd as H
    from oracle import oracle as O
    hip = H.lib()                                     # libhiphuff.so (HIP runtime via torch)
    ref = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libhuffref.so"))
    ref.newDecoder.restype = C.c_void_p
    ref.newDecoder.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p]
    ref.loadTestData.restype = C.c_void_p
    ref.loadTestData.argtypes = [C.c_char_p, C.c_char_p]
    ref.evaluate.restype = C.c_double
    ref.evaluate.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    ref.evalandshow.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    libc = C.CDLL(None)
    fn = C.cast(hip.hipHuffApproach, C.c_void_p)
    dec = ref.newDecoder(fn, None, b"hip")
    tmp = tempfile.mkdtemp(prefix="hh_harness_")
    for name in names:
        huff = os.path.join(ROOT, "files", name + ".huff")
        orig = os.path.join(ROOT, "files", name)
        if not os.path.exists(orig):
            data = O.OracleHuff.load(huff).chain_decode().tobytes()
            if hashlib.sha256(data).hexdigest() != DIGESTS[name]:
                raise SystemExit(f"regenerated {name} does not match its recorded sha256")
            orig = os.path.join(tmp, name)
            with open(orig, "wb") as f:
                f.write(data)
            os.symlink(huff, orig + ".huff")
        td = ref.loadTestData(orig.encode(), name.encode())
        ref.evalandshow(C.c_void_p(dec), C.c_void_p(td), 1)
        libc.fflush(None)
    sys.stdout.flush()


if __name__ == "__main__":
    main(sys.argv[1:])
