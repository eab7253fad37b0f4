"""Regenerate the originals the reference tree omits (kjv.txt, E.coli) next
to the shipped fixtures, for the CLI's byte-checked graph runs.

    python tools/regen_files.py OUTDIR

OUTDIR receives a symlink to every file under files/ and, for each missing
original, the text decoded from its .huff by the oracle's serial decoder,
checked against the sha256 digest recorded in BASELINE.md before it is
written (the same recipe as tests/harness_ref.py).  Then

    build/HuffFramework graph2 --files OUTDIR

byte-compares every prefix against the original, as the reference's
graphtest does (framework/mainrun.c:387-410 -> evaluate(d, &reducedTd, 1),
decodeUtil.c:47-52).  Test/tool infrastructure: the oracle is the checker
here, never the decoder being measured.
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DIGESTS = {   # BASELINE.md / SURVEY.md 8(c)
    "kjv.txt": "e4e21579f6360b35e66dc97b67cd732a3f759623e41e4e077bec039eeb79fd0a",
    "E.coli": "9125dfd87315961ef4286f3856098069e050cc3a2abe65735fe43e69d1996f40",
}


def regen(outdir: str, names=("kjv.txt", "E.coli")) -> str:
    from oracle import oracle as O
    src = os.path.join(ROOT, "files")
    os.makedirs(outdir, exist_ok=True)
    for f in os.listdir(src):
        dst = os.path.join(outdir, f)
        if not os.path.lexists(dst):
            os.symlink(os.path.join(src, f), dst)
    for name in names:
        dst = os.path.join(outdir, name)
        if os.path.exists(dst):
            continue
        data = O.OracleHuff.load(os.path.join(src, name + ".huff")).chain_decode().tobytes()
        if hashlib.sha256(data).hexdigest() != DIGESTS[name]:
            raise SystemExit(f"regenerated {name} does not match its recorded sha256")
        with open(dst, "wb") as f:
            f.write(data)
    return outdir


if __name__ == "__main__":
    print(regen(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "files_full")))
