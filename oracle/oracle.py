"""ctypes bindings to the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  Two backends:

* ``liboracle.so`` -- the clean-room C restatement (oracle/hh_oracle.c).
* ``_ref/libhuffref.so`` -- the reference's own C sources compiled in place by
  oracle/Makefile (present only where it was built; it travels to the GPU box
  as a prebuilt .so, the reference tree itself does not).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None


class _OrHuff(C.Structure):
    _fields_ = [("bits", C.c_int64), ("uncompressedsize", C.c_int64),
                ("nodes", C.c_int32),
                ("izero", C.POINTER(C.c_int32)), ("ione", C.POINTER(C.c_int32)),
                ("sym", C.POINTER(C.c_uint8)), ("data", C.POINTER(C.c_uint8))]


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(path)
        P = C.POINTER
        L.or_load_huff.argtypes = [C.c_char_p, P(_OrHuff)]
        L.or_free_huff.argtypes = [P(_OrHuff)]
        for name in ("or_simple_decode", "or_chain_decode"):
            fn = getattr(L, name)
            fn.argtypes = [P(_OrHuff), C.c_void_p, C.c_int64]
            fn.restype = C.c_int64
        L.or_lin_decode.argtypes = [P(_OrHuff), C.c_int, C.c_void_p, C.c_int64]
        L.or_lin_decode.restype = C.c_int64
        L.or_pes.argtypes = [P(_OrHuff), C.c_void_p, C.c_void_p, C.c_void_p,
                             C.c_void_p, P(C.c_int32)]
        L.or_pes.restype = C.c_int64
        L.or_now.restype = C.c_double
        _LIB = L
    return _LIB


@dataclass
class Huff:
    """A .huff file as numpy arrays (izero/ione/sym per node, payload)."""
    bits: int
    uncompressedsize: int
    izero: np.ndarray
    ione: np.ndarray
    sym: np.ndarray
    data: np.ndarray  # payload bytes, no padding

    @property
    def nodes(self) -> int:
        return int(self.izero.shape[0])


class OracleHuff:
    """Owns an or_huff loaded (or built) in C memory."""

    def __init__(self, h: _OrHuff, owned: bool):
        self._h = h
        self._owned = owned
        self._keep = []

    @classmethod
    def load(cls, path: str) -> "OracleHuff":
        h = _OrHuff()
        rc = lib().or_load_huff(path.encode(), C.byref(h))
        if rc != 0:
            raise ValueError(f"or_load_huff({path}) failed: {rc}")
        return cls(h, True)

    @classmethod
    def from_arrays(cls, hf: Huff) -> "OracleHuff":
        h = _OrHuff()
        iz = np.ascontiguousarray(hf.izero, dtype=np.int32)
        io = np.ascontiguousarray(hf.ione, dtype=np.int32)
        sy = np.ascontiguousarray(hf.sym, dtype=np.uint8)
        pad = np.zeros(len(hf.data) + 16, dtype=np.uint8)
        pad[: len(hf.data)] = hf.data
        h.bits, h.uncompressedsize, h.nodes = hf.bits, hf.uncompressedsize, len(iz)
        h.izero = iz.ctypes.data_as(C.POINTER(C.c_int32))
        h.ione = io.ctypes.data_as(C.POINTER(C.c_int32))
        h.sym = sy.ctypes.data_as(C.POINTER(C.c_uint8))
        h.data = pad.ctypes.data_as(C.POINTER(C.c_uint8))
        o = cls(h, False)
        o._keep = [iz, io, sy, pad]
        return o

    def __del__(self):
        if getattr(self, "_owned", False) and _LIB is not None:
            _LIB.or_free_huff(C.byref(self._h))
            self._owned = False

    @property
    def bits(self) -> int:
        return int(self._h.bits)

    @property
    def uncompressedsize(self) -> int:
        return int(self._h.uncompressedsize)

    def _decode(self, fn, cap):
        out = np.zeros(cap, dtype=np.uint8)
        n = fn(C.byref(self._h), out.ctypes.data, cap)
        if n < 0:
            raise RuntimeError("oracle decode failed")
        return out[:n]

    def simple_decode(self) -> np.ndarray:
        return self._decode(lib().or_simple_decode, self.bits + 1)

    def chain_decode(self) -> np.ndarray:
        return self._decode(lib().or_chain_decode, self.bits + 1)

    def lin_decode(self, jumpbits: int) -> np.ndarray:
        cap = self.uncompressedsize + 64
        out = np.zeros(cap, dtype=np.uint8)
        n = lib().or_lin_decode(C.byref(self._h), jumpbits, out.ctypes.data, cap)
        if n < 0:
            raise RuntimeError("or_lin_decode failed")
        return out[: min(n, self.uncompressedsize)]

    def pes(self):
        """Returns dict of the pes stage arrays (small inputs only)."""
        B = self.bits
        bitdecode = np.zeros(B, np.uint8)
        steps = np.zeros(25 * B, np.int32)
        idx = np.zeros(B, np.int32)
        result = np.zeros(B, np.uint8)
        nl = C.c_int32(0)
        n = lib().or_pes(C.byref(self._h), bitdecode.ctypes.data, steps.ctypes.data,
                         idx.ctypes.data, result.ctypes.data, C.byref(nl))
        if n < 0:
            raise RuntimeError("or_pes failed")
        return dict(bitdecode=bitdecode, steps=steps.reshape(25, B)[: nl.value + 1],
                    bitsindex=idx, result=result[:n], nlevels=nl.value)


def now() -> float:
    return lib().or_now()


# ---------------------------------------------------------------------------
# The reference's own C code (oracle/_ref/libhuffref.so), when built.
# ---------------------------------------------------------------------------
class _RefNode(C.Structure):
    _fields_ = [("sym", C.c_ubyte), ("izero", C.c_int), ("ione", C.c_int)]


class _RefCD(C.Structure):   # huffdata.h:26-32
    _fields_ = [("bits", C.c_int), ("nodes", C.c_int), ("uncompressedsize", C.c_int),
                ("tree", C.POINTER(_RefNode)), ("data", C.POINTER(C.c_ubyte))]


class _RefUCD(C.Structure):  # huffdata.h:34-37
    _fields_ = [("uncompressedsize", C.c_int), ("data", C.POINTER(C.c_ubyte))]


def ref_available() -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", "libhuffref.so"))


def ref() -> C.CDLL:
    global _REF
    if _REF is None:
        L = C.CDLL(os.path.join(HERE, "_ref", "libhuffref.so"))
        L.loadHuffFile.argtypes = [C.c_char_p]
        L.loadHuffFile.restype = C.POINTER(_RefCD)
        L.freeCompressedData.argtypes = [C.POINTER(_RefCD)]
        sig = [C.POINTER(_RefCD), C.POINTER(_RefUCD), C.c_void_p]
        for name in ("linApproach", "jumptableApproach", "simpleDecode", "pesApproach",
                     "decodeBigtableMultiSym", "decodeBigtableSimple"):
            getattr(L, name).argtypes = sig
        _REF = L
    return _REF


class RefHuff:
    """A .huff loaded by the reference's own loadHuffFile (huffdata.c:27)."""

    def __init__(self, path: str):
        self.cd = ref().loadHuffFile(path.encode())
        if not self.cd:
            raise ValueError(path)

    def __del__(self):
        if getattr(self, "cd", None) and _REF is not None and getattr(self, "_owned", True):
            _REF.freeCompressedData(self.cd)
        self.cd = None

    @classmethod
    def from_arrays(cls, izero, ione, sym, data, bits: int, uncompressedsize: int = 0) -> "RefHuff":
        """An in-memory CompressedData (huffdata.h:26-32) for the reference's
        decoders: the tree as its HuffNode array, the payload followed by the
        3 zero bytes loadHuffFile appends (huffdata.c:55-64)."""
        self = cls.__new__(cls)
        n = len(izero)
        self._nodes = (_RefNode * n)(*[_RefNode(int(sym[i]) & 255, int(izero[i]), int(ione[i])) for i in range(n)])
        nb = (bits + 7) // 8
        self._data = np.zeros(nb + 3, dtype=np.uint8)
        self._data[:nb] = np.asarray(data, np.uint8)[:nb]
        self._cd = _RefCD(int(bits), n, int(uncompressedsize or bits),
                          C.cast(self._nodes, C.POINTER(_RefNode)),
                          self._data.ctypes.data_as(C.POINTER(C.c_ubyte)))
        self.cd = C.pointer(self._cd)
        self._owned = False
        return self

    @property
    def uncompressedsize(self) -> int:
        return self.cd.contents.uncompressedsize

    def run(self, name: str, jumpbits: int | None = None) -> np.ndarray:
        n = self.uncompressedsize
        buf = np.zeros(n + 64, dtype=np.uint8)
        ucd = _RefUCD(n, buf.ctypes.data_as(C.POINTER(C.c_ubyte)))
        param = C.byref(C.c_int(jumpbits)) if jumpbits is not None else None
        getattr(ref(), name)(self.cd, C.byref(ucd), param)
        return buf[: ucd.uncompressedsize]
