"""Regenerate tests/golden/*.json from the oracle (run from the repo root).

hello_pes.json is the known-answer trace of SURVEY.md A.1: every stage array
of the reference's pes pipeline (framework/pes.c) on files/hello.huff.  The
same trace was recorded from the reference's own pes.c in the survey
container; test_oracle.py pins the oracle to it and, where oracle/_ref is
built, to the reference binary itself.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402


def main():
    h = O.OracleHuff.load(os.path.join(ROOT, "files", "hello.huff"))
    p = h.pes()
    g = {
        "file": "files/hello.huff",
        "bits": h.bits,
        "nlevels": p["nlevels"],
        "levels": [list(map(int, row)) for row in p["steps"]],
        "bitdecode": list(map(int, p["bitdecode"])),
        "bitsindex": list(map(int, p["bitsindex"])),
        "result": bytes(p["result"]).decode(),
        "digests": {
            "kjv.txt": "e4e21579f6360b35e66dc97b67cd732a3f759623e41e4e077bec039eeb79fd0a",
            "E.coli": "9125dfd87315961ef4286f3856098069e050cc3a2abe65735fe43e69d1996f40",
        },
    }
    with open(os.path.join(ROOT, "tests", "golden", "hello_pes.json"), "w") as f:
        json.dump(g, f, indent=1)


if __name__ == "__main__":
    main()
