"""hiphuff -- MI355X-native parallel Huffman decoder (Python host binding).

A thin ctypes layer over the C ABI in ``include/hiphuff.h`` (the library
``libhiphuff.so`` in this package directory, built by the top-level
Makefile).  The decode itself always runs in the HIP kernels; there is no CPU
fallback in this package -- if the library (or a GPU) is missing, the calls
raise.

Mirrors the reference's plugin interface (framework/decodeUtil.h:14-19): a
``Decoder`` is the device state behind one decoder function, ``decode_host``
is the evaluate()-timed scope (H2D + decode + D2H, decodeUtil.c:41-43) and
``decode_device`` is the HBM-resident hot path.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# HIPHUFF_LIB overrides the library (diagnostic builds, e.g. build/libhiphuff_stamps.so)
LIB_PATH = os.environ.get("HIPHUFF_LIB") or os.path.join(HERE, "libhiphuff.so")
PAYLOAD_PAD = 64   # HH_PAYLOAD_PAD

_ERRORS = {
    0: "ok", -1: "bad argument", -2: "i/o error", -3: "not a HUFF/HUFX file",
    -4: "invalid code tree", -5: "output buffer too small", -6: "HIP runtime error",
    -7: "out of memory", -8: "internal error", -9: "in-kernel wait timed out",
    -10: "unsupported input",
}


class HipHuffError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {_ERRORS.get(status, status)} ({status})")


class _Huff(C.Structure):
    _fields_ = [("nodes", C.c_int32), ("izero", C.POINTER(C.c_int32)),
                ("ione", C.POINTER(C.c_int32)), ("sym", C.POINTER(C.c_uint8)),
                ("bits", C.c_uint64), ("uncompressedsize", C.c_uint64),
                ("data", C.POINTER(C.c_uint8)), ("wide", C.c_int)]


class _Tree(C.Structure):
    _fields_ = [("nodes", C.c_int32), ("izero", C.c_void_p), ("ione", C.c_void_p),
                ("sym", C.c_void_p)]


class _TreeInfo(C.Structure):
    _fields_ = [("reachable", C.c_int32), ("leaves", C.c_int32), ("minlen", C.c_int32),
                ("maxlen", C.c_int32), ("len_gcd", C.c_int32)]


class _Config(C.Structure):
    _fields_ = [("device", C.c_int), ("lane_bits", C.c_int), ("flags", C.c_int)]


class _Stats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_sync", C.c_double), ("ms_scan", C.c_double),
                ("ms_emit", C.c_double), ("out_len", C.c_uint64), ("lanes", C.c_uint64),
                ("repairs", C.c_uint64), ("exact_fallback", C.c_int), ("fixed_length", C.c_int),
                ("state_machine", C.c_int)]


class _Range(C.Structure):
    _fields_ = [("bits_avail", C.c_uint64), ("ntiles", C.c_uint64), ("prologue", C.c_uint64),
                ("in_state", C.c_uint32)]


class _RangeOut(C.Structure):
    _fields_ = [("out_len", C.c_uint64), ("leave_state", C.c_uint32), ("const_seen", C.c_uint32),
                ("entry_state", C.c_uint32), ("entry_exact", C.c_uint32)]


FLAG_FORCE_EXACT = 1
FLAG_FORCE_SEGMENT = 2
FLAG_NO_FIXED = 4     # HH_FLAG_NO_FIXED: fixed-length codes through the general pipeline too
FLAG_LEGACY = 8       # HH_FLAG_LEGACY: round 2's pipeline instead of the state-machine decode
FLAG_PHASE_TIMING = 16  # HH_FLAG_PHASE_TIMING: events between the kernels (ms_sync/scan/emit)
FLAG_KEEP_HOST_PINNED = 32  # HH_FLAG_KEEP_HOST_PINNED: decode_host keeps the caller's buffers page-locked
FLAG_TWO_PASS = 64    # HH_FLAG_TWO_PASS: the state machine's two-pass form instead of its single pass
_lib_handle: Optional[C.CDLL] = None

# exported symbols and their ctypes signatures; tests check every one of these
# against include/hiphuff.h
_SIGS = {
    "hh_strerror": ([C.c_int], C.c_char_p),
    "hh_tree_check": ([C.POINTER(_Tree), C.POINTER(_TreeInfo)], C.c_int),
    "hh_huff_load": ([C.c_char_p, C.POINTER(_Huff)], C.c_int),
    "hh_huff_save": ([C.c_char_p, C.POINTER(_Huff)], C.c_int),
    "hh_huff_free": ([C.POINTER(_Huff)], None),
    "hh_huff_tree": ([C.POINTER(_Huff)], _Tree),
    "hh_encode_bound": ([C.POINTER(_Tree), C.c_uint64], C.c_uint64),
    "hh_encode": ([C.POINTER(_Tree), C.c_void_p, C.c_uint64, C.c_void_p,
                   C.POINTER(C.c_uint64)], C.c_int),
    "hh_encode_device": ([C.POINTER(_Tree), C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                          C.POINTER(C.c_uint64), C.c_void_p], C.c_int),
    "hh_encoder_create": ([C.POINTER(C.c_void_p), C.c_int], C.c_int),
    "hh_encoder_destroy": ([C.c_void_p], None),
    "hh_encoder_encode": ([C.c_void_p, C.POINTER(_Tree), C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                           C.POINTER(C.c_uint64), C.c_void_p], C.c_int),
    "hh_decoder_create": ([C.POINTER(C.c_void_p), C.POINTER(_Config)], C.c_int),
    "hh_decoder_destroy": ([C.c_void_p], None),
    "hh_decoder_set_tree": ([C.c_void_p, C.POINTER(_Tree)], C.c_int),
    "hh_decoder_stats": ([C.c_void_p, C.POINTER(_Stats)], C.c_int),
    "hh_decode_device": ([C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                          C.POINTER(C.c_uint64), C.c_void_p], C.c_int),
    "hh_decode_device_async": ([C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                C.POINTER(C.c_uint64), C.c_void_p], C.c_int),
    "hh_decode_wait": ([C.c_void_p], C.c_int),
    "hh_decoder_tile_bits": ([C.c_void_p, C.POINTER(C.c_uint64)], C.c_int),
    "hh_decode_device_range": ([C.c_void_p, C.c_void_p, C.POINTER(_Range), C.c_void_p,
                                C.c_uint64, C.POINTER(_RangeOut), C.c_void_p], C.c_int),
    "hh_decode_device_range_async": ([C.c_void_p, C.c_void_p, C.POINTER(_Range), C.c_void_p,
                                      C.c_uint64, C.POINTER(_RangeOut), C.c_void_p], C.c_int),
    "hh_decoder_release_host": ([C.c_void_p], C.c_int),
    "hh_decode_host": ([C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                        C.POINTER(C.c_uint64)], C.c_int),
    "hh_copy_device": ([C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p,
                        C.POINTER(C.c_float)], C.c_int),
    "hh_stage_initbitsindex": ([C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p], C.c_int),
    "hh_stage_decodeallbits": ([C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                C.c_void_p], C.c_int),
    "hh_stage_makebigtable": ([C.c_void_p, C.c_int64, C.c_void_p, C.c_int32,
                               C.POINTER(C.c_int32), C.c_void_p], C.c_int),
    "hh_stage_calcbitsindex": ([C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32,
                                C.c_int32, C.c_void_p], C.c_int),
    "hh_stage_calcresult": ([C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                             C.c_void_p], C.c_int),
    "hh_stage_findmax": ([C.c_void_p, C.c_int64, C.c_void_p, C.POINTER(C.c_int32),
                          C.c_void_p], C.c_int),
    "hh_stage_pipeline": ([C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_uint64,
                           C.POINTER(C.c_uint64), C.c_void_p], C.c_int),
    "hipHuffApproach": ([C.c_void_p, C.c_void_p, C.c_void_p], None),
    "hh_debug_counters": ([C.c_void_p, C.c_void_p], C.c_int),
    "hh_debug_fsm": ([C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
}


def lib() -> C.CDLL:
    """The HIP library; raises if it was not built (no silent fallback)."""
    global _lib_handle
    if _lib_handle is None:
        # One HIP runtime per process: torch ships its own libamdhip64.so.7.
        # Loading torch first lets libhiphuff.so bind to that same runtime
        # (same soname), so device pointers and streams are shared with torch.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        # every declared symbol must be there; only an explicit A/B build
        # of an older revision (HIPHUFF_AB_BUILD=1, tools/mkrev.sh) may lack
        # some -- those are named on stderr and left unbound
        ab = os.environ.get("HIPHUFF_AB_BUILD") == "1"
        skipped = []
        for name, (args, res) in _SIGS.items():
            if ab and not hasattr(L, name):
                skipped.append(name)
                continue
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if skipped:
            import sys
            print(f"hiphuff: {LIB_PATH} (HIPHUFF_AB_BUILD) lacks {', '.join(skipped)}", file=sys.stderr)
        _lib_handle = L
    return _lib_handle


def _check(rc: int, what: str):
    if rc != 0:
        raise HipHuffError(rc, what)


@dataclass
class HuffFile:
    """A .huff container (HUFF or 64-bit HUFX), huffdata.c:27-68."""
    izero: np.ndarray
    ione: np.ndarray
    sym: np.ndarray
    bits: int
    uncompressedsize: int
    data: np.ndarray       # payload + PAYLOAD_PAD zero bytes

    @property
    def nodes(self) -> int:
        return int(self.izero.shape[0])

    @property
    def payload(self) -> np.ndarray:
        return self.data[: (self.bits + 7) // 8]

    @classmethod
    def load(cls, path: str) -> "HuffFile":
        h = _Huff()
        _check(lib().hh_huff_load(path.encode(), C.byref(h)), f"load {path}")
        try:
            n = h.nodes
            iz = np.ctypeslib.as_array(h.izero, shape=(n,)).copy()
            io = np.ctypeslib.as_array(h.ione, shape=(n,)).copy()
            sy = np.ctypeslib.as_array(h.sym, shape=(n,)).copy()
            nb = (h.bits + 7) // 8 + PAYLOAD_PAD
            data = np.ctypeslib.as_array(h.data, shape=(nb,)).copy()
            return cls(iz, io, sy, int(h.bits), int(h.uncompressedsize), data)
        finally:
            lib().hh_huff_free(C.byref(h))

    def save(self, path: str, wide: bool = False):
        keep = [np.ascontiguousarray(self.izero, np.int32),
                np.ascontiguousarray(self.ione, np.int32),
                np.ascontiguousarray(self.sym, np.uint8),
                np.ascontiguousarray(self.data, np.uint8)]
        h = _Huff(self.nodes, keep[0].ctypes.data_as(C.POINTER(C.c_int32)),
                  keep[1].ctypes.data_as(C.POINTER(C.c_int32)),
                  keep[2].ctypes.data_as(C.POINTER(C.c_uint8)), self.bits,
                  self.uncompressedsize, keep[3].ctypes.data_as(C.POINTER(C.c_uint8)),
                  int(wide))
        _check(lib().hh_huff_save(path.encode(), C.byref(h)), f"save {path}")

    def tree(self) -> "Tree":
        return Tree(self.izero, self.ione, self.sym)


class Tree:
    """Code tree in the reference's node layout (huffdata.h:12-16), SoA."""

    def __init__(self, izero, ione, sym):
        self.izero = np.ascontiguousarray(izero, np.int32)
        self.ione = np.ascontiguousarray(ione, np.int32)
        self.sym = np.ascontiguousarray(sym, np.uint8)
        self._c = _Tree(len(self.izero), self.izero.ctypes.data, self.ione.ctypes.data,
                        self.sym.ctypes.data)

    def info(self) -> dict:
        inf = _TreeInfo()
        _check(lib().hh_tree_check(C.byref(self._c), C.byref(inf)), "tree check")
        return {k: getattr(inf, k) for k, _ in _TreeInfo._fields_}

    def encode(self, syms: np.ndarray) -> tuple[np.ndarray, int]:
        """Pack symbols LSB-first with this tree's codes -> (payload+pad, bits)."""
        syms = np.ascontiguousarray(syms, np.uint8)
        bound = lib().hh_encode_bound(C.byref(self._c), len(syms))
        if bound == 0:
            raise HipHuffError(-4, "encode bound")
        out = np.zeros(bound + PAYLOAD_PAD, np.uint8)
        bits = C.c_uint64(0)
        _check(lib().hh_encode(C.byref(self._c), syms.ctypes.data, len(syms), out.ctypes.data,
                               C.byref(bits)), "encode")
        nb = (bits.value + 7) // 8
        return out[: nb + PAYLOAD_PAD].copy(), int(bits.value)


def encode_device(tree: "Tree", syms, out, stream=None) -> int:
    """Pack torch uint8 CUDA symbols with tree's codes into the torch uint8
    CUDA tensor out (hh_encode_device; out must hold the stream rounded up
    to 32-bit words, plus PAYLOAD_PAD for a decode).  Returns the bits."""
    import torch
    assert syms.is_cuda and out.is_cuda and syms.dtype == torch.uint8 and out.dtype == torch.uint8
    bits = C.c_uint64(0)
    _check(lib().hh_encode_device(C.byref(tree._c), syms.data_ptr(), syms.numel(), out.data_ptr(), out.numel(),
                                  C.byref(bits), stream.cuda_stream if stream is not None else None),
           "encode_device")
    return int(bits.value)


class Encoder:
    """A device encoder (hh_encoder_*): its own workspace, so that encoders
    on different streams (or threads) encode at once."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        _check(lib().hh_encoder_create(C.byref(self._h), device), "encoder create")

    def encode(self, tree: "Tree", syms, out, stream=None) -> int:
        """encode_device on this encoder."""
        import torch
        assert syms.is_cuda and out.is_cuda and syms.dtype == torch.uint8 and out.dtype == torch.uint8
        bits = C.c_uint64(0)
        _check(lib().hh_encoder_encode(self._h, C.byref(tree._c), syms.data_ptr(), syms.numel(), out.data_ptr(),
                                       out.numel(), C.byref(bits), stream.cuda_stream if stream is not None else None),
               "encoder_encode")
        return int(bits.value)

    def close(self):
        if self._h:
            lib().hh_encoder_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def copy_device(src, dst, nt: bool = False, stream=None) -> float:
    """hh_copy_device on torch uint8 CUDA tensors (the same number of bytes,
    a multiple of 16): the streaming-copy reference; returns its device ms."""
    import torch
    assert src.is_cuda and dst.is_cuda and src.numel() == dst.numel()
    ms = C.c_float(0.0)
    s = stream if stream is not None else torch.cuda.current_stream(src.device)
    _check(lib().hh_copy_device(src.data_ptr(), dst.data_ptr(), src.numel(), int(nt), s.cuda_stream,
                                C.byref(ms)), "copy_device")
    return float(ms.value)


class RangeResult:
    """The hh_range_out of an asynchronous segment decode (valid once checked)."""

    def __init__(self):
        self._ro = _RangeOut()

    def as_dict(self) -> dict:
        ro = self._ro
        return {"out_len": int(ro.out_len), "leave_state": int(ro.leave_state),
                "const_seen": bool(ro.const_seen), "entry_state": int(ro.entry_state),
                "entry_exact": bool(ro.entry_exact)}


class Decoder:
    """Device decoder: tables + workspace on one GPU (hh_decoder_*)."""

    def __init__(self, device: int = 0, lane_bits: int = 0, flags: int = 0):
        self._h = C.c_void_p()
        cfg = _Config(device, lane_bits, flags)
        _check(lib().hh_decoder_create(C.byref(self._h), C.byref(cfg)), "decoder create")
        self.device = device
        self.flags = flags
        self._tree = None
        self._pending = []          # buffers of asynchronous decodes, kept alive until wait()
        self._pinned = None         # (payload, out) FLAG_KEEP_HOST_PINNED keeps registered

    def close(self):
        if self._h:
            lib().hh_decoder_destroy(self._h)   # (waits for an asynchronous decode still running)
            self._h = C.c_void_p()
        self._pending = []
        self._pinned = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_tree(self, tree: Tree):
        _check(lib().hh_decoder_set_tree(self._h, C.byref(tree._c)), "set tree")
        self._tree = tree

    def stats(self) -> dict:
        st = _Stats()
        _check(lib().hh_decoder_stats(self._h, C.byref(st)), "stats")
        return {k: getattr(st, k) for k, _ in _Stats._fields_}

    def decode_host(self, payload: np.ndarray, bits: int, cap: int,
                    out: Optional[np.ndarray] = None) -> np.ndarray:
        """The evaluate() scope: host payload in, host symbols out.  `out`
        (uint8, >= cap) may be the caller's buffer, allocated and touched
        beforehand as evaluate() does (decodeUtil.c:37-38, 55)."""
        keep = bool(self.flags & FLAG_KEEP_HOST_PINNED)
        given = payload
        payload = np.ascontiguousarray(payload, np.uint8)
        # (copied: the caller's memory is not what gets registered -- a new
        # view of the same memory is fine, so the data pointers are compared)
        copied = not (isinstance(given, np.ndarray)
                      and given.__array_interface__["data"][0] == payload.__array_interface__["data"][0])
        if keep and (out is None or copied):
            # the decoder keeps both buffers registered after the call: they
            # must be the caller's own arrays, alive until release_host()
            # (a temporary freed after the call could be reallocated at the
            # same address and pass for the registered one)
            raise ValueError("FLAG_KEEP_HOST_PINNED: pass a contiguous uint8 payload and an `out` buffer")
        if out is None:
            out = np.zeros(max(cap, 1), np.uint8)
        assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size >= cap
        n = C.c_uint64(0)
        _check(lib().hh_decode_host(self._h, payload.ctypes.data, bits, out.ctypes.data, cap,
                                    C.byref(n)), "decode_host")
        if keep:
            self._pinned = (given, out)       # (alive while registered)
        return out[: n.value]

    def release_host(self) -> None:
        """hh_decoder_release_host: unpin the buffers FLAG_KEEP_HOST_PINNED kept."""
        _check(lib().hh_decoder_release_host(self._h), "release_host")
        self._pinned = None

    def decode_device_ptr(self, d_data: int, bits: int, d_out: int, cap: int,
                          stream: int = 0) -> int:
        n = C.c_uint64(0)
        _check(lib().hh_decode_device(self._h, d_data, bits, d_out, cap, C.byref(n),
                                      stream or None), "decode_device")
        return int(n.value)

    def decode_device(self, data, bits: int, out, stream=None) -> int:
        """Decode torch uint8 CUDA tensors (data holds payload + pad)."""
        import torch
        assert data.is_cuda and out.is_cuda and data.dtype == torch.uint8
        assert data.numel() >= (bits + 7) // 8 + PAYLOAD_PAD
        s = stream if stream is not None else torch.cuda.current_stream(data.device)
        return self.decode_device_ptr(data.data_ptr(), bits, out.data_ptr(), out.numel(),
                                      s.cuda_stream)

    def decode_device_async(self, data, bits: int, out, stream=None) -> "C.c_uint64":
        """hh_decode_device_async on torch tensors: enqueues the decode and
        returns a c_uint64 that holds its length once checked (by the next
        asynchronous decode or by wait()).  data, out and the returned
        object must live until wait() returns."""
        import torch
        assert data.is_cuda and out.is_cuda and data.dtype == torch.uint8
        assert data.numel() >= (bits + 7) // 8 + PAYLOAD_PAD
        s = stream if stream is not None else torch.cuda.current_stream(data.device)
        n = C.c_uint64(0)
        self._pending.append((data, out, n))
        _check(lib().hh_decode_device_async(self._h, data.data_ptr(), bits, out.data_ptr(), out.numel(),
                                            C.byref(n), s.cuda_stream), "decode_device_async")
        return n

    def wait(self) -> None:
        """hh_decode_wait: every asynchronous decode checked; raises the first
        failure among them."""
        rc = lib().hh_decode_wait(self._h)
        self._pending = []
        _check(rc, "decode_wait")

    def tile_bits(self) -> int:
        """Bits per tile for the current tree (segments are whole tiles)."""
        tb = C.c_uint64(0)
        _check(lib().hh_decoder_tile_bits(self._h, C.byref(tb)), "tile_bits")
        return int(tb.value)

    def decode_range_ptr(self, d_data: int, bits_avail: int, ntiles: int, in_state: int,
                         d_out: int, cap: int, stream: int = 0, prologue: int = 0) -> dict:
        """One segment (hh_decode_device_range): tiles [0, ntiles) of the
        bits at d_data, entered in state in_state; the first `prologue`
        tiles only locate the entry of tile `prologue`."""
        rg = _Range(bits_avail, ntiles, prologue, in_state)
        ro = _RangeOut()
        _check(lib().hh_decode_device_range(self._h, d_data, C.byref(rg), d_out, cap,
                                            C.byref(ro), stream or None), "decode_range")
        return {"out_len": int(ro.out_len), "leave_state": int(ro.leave_state),
                "const_seen": bool(ro.const_seen), "entry_state": int(ro.entry_state),
                "entry_exact": bool(ro.entry_exact)}

    def decode_range_async_ptr(self, d_data: int, bits_avail: int, ntiles: int, in_state: int,
                               d_out: int, cap: int, stream: int = 0, prologue: int = 0) -> "RangeResult":
        """hh_decode_device_range_async: enqueues the segment's decode and
        returns a RangeResult whose fields are valid once the decode has been
        checked (by the next asynchronous decode on this decoder, or wait())."""
        rg = _Range(bits_avail, ntiles, prologue, in_state)
        r = RangeResult()
        self._pending.append(r)
        _check(lib().hh_decode_device_range_async(self._h, d_data, C.byref(rg), d_out, cap,
                                                  C.byref(r._ro), stream or None), "decode_range_async")
        return r

    def stage_pipeline_ptr(self, d_data: int, bits: int, d_out: int, cap: int,
                           stream: int = 0) -> int:
        n = C.c_uint64(0)
        _check(lib().hh_stage_pipeline(self._h, d_data, bits, d_out, cap, C.byref(n),
                                       stream or None), "stage_pipeline")
        return int(n.value)


def decode_file(path: str, device: int = 0) -> np.ndarray:
    """Load a .huff and decode it on the GPU (host-to-host)."""
    hf = HuffFile.load(path)
    dec = Decoder(device)
    try:
        dec.set_tree(hf.tree())
        return dec.decode_host(hf.payload, hf.bits, hf.bits + 1)
    finally:
        dec.close()
