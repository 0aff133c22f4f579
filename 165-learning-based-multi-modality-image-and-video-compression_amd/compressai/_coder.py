"""ctypes binding of libcai_coder.so (include/cai_coder.h): quantized CDFs and rANS.

Host code, like the reference's pybind11 modules ``compressai._CXX`` and
``compressai.ans`` (cpp_exts/ops/ops.cpp, cpp_exts/rans/rans_interface.cpp).
Errors follow the reference's convention: argument errors raise ValueError
(std::domain_error there), a missing library raises RuntimeError.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_float, c_int, c_int32, c_int64, c_void_p
from typing import Optional, Sequence

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("CAI_CODER_LIB", os.path.join(_PKG_ROOT, "lib", "libcai_coder.so"))

CAI_OK, CAI_EINVAL, CAI_EWORKSPACE = 0, 1, 3


class RansTables(Structure):
    _fields_ = [("cdfs", c_void_p), ("cdf_stride", c_int64), ("cdf_sizes", c_void_p), ("offsets", c_void_p),
                ("n_cdfs", c_int32)]


_P, _I64 = c_void_p, c_int64
_T = POINTER(RansTables)
SIGNATURES = {
    "cai_coder_last_error": (c_char_p, []),
    "cai_coder_abi_count": (c_int, []),
    "cai_pmf_to_quantized_cdf": (c_int, [_P, c_int32, c_int32, _P]),
    "cai_pmf_to_quantized_cdf_rows": (c_int, [_P, _I64, _P, c_int32, c_int32, _P, _I64, c_int32]),
    "cai_rans_max_bytes": (_I64, [_I64]),
    "cai_rans_encode": (c_int, [_P, _P, _I64, _T, _P, _I64, _P]),
    "cai_rans_encode_batch": (c_int, [c_int32, _P, _P, _P, _T, _P, _P, _P, c_int32]),
    "cai_rans_decode": (c_int, [_P, _I64, _P, _I64, _T, _P]),
    "cai_rans_decode_batch": (c_int, [c_int32, _P, _P, _P, _P, _P, _T, _P, c_int32]),
    "cai_rans_buffered_create": (c_void_p, []),
    "cai_rans_buffered_destroy": (None, [_P]),
    "cai_rans_buffered_encode": (c_int, [_P, _P, _P, _I64, _T]),
    "cai_rans_buffered_max_bytes": (_I64, [_P]),
    "cai_rans_buffered_flush": (c_int, [_P, _P, _I64, _P]),
    "cai_rans_decoder_create": (c_void_p, []),
    "cai_rans_decoder_destroy": (None, [_P]),
    "cai_rans_decoder_set_stream": (c_int, [_P, _P, _I64]),
    "cai_rans_decoder_decode_stream": (c_int, [_P, _P, _I64, _T, _P]),
}
_RAW = {"cai_coder_last_error", "cai_coder_abi_count", "cai_rans_max_bytes", "cai_rans_buffered_create",
        "cai_rans_buffered_destroy", "cai_rans_buffered_max_bytes", "cai_rans_decoder_create",
        "cai_rans_decoder_destroy"}


def default_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


class _Lib:
    def __init__(self):
        self._lib = None

    def load(self):
        if self._lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libcai_coder.so not found at {LIB_PATH}: build it with "
                                   "`python -c 'import __graft_entry__ as g; g.build()'`")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            self._lib = lib
        return self._lib

    def __getattr__(self, name):
        fn = getattr(self.load(), name)
        if name in _RAW:
            return fn

        def call(*args):
            rc = fn(*args)
            if rc != CAI_OK:
                msg = self.load().cai_coder_last_error().decode(errors="replace")
                raise ValueError(f"{name}: {msg}")
            return rc
        return call


lib = _Lib()


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else c_void_p(a.ctypes.data)


def i32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


class Tables:
    """CDF table set (cdfs [n][stride], sizes [n], offsets [n]) kept alive for the C calls."""

    def __init__(self, cdfs, cdf_sizes, offsets):
        if isinstance(cdfs, np.ndarray) and cdfs.ndim == 2:
            arr = i32(cdfs)
        else:
            rows = [list(r) for r in cdfs]
            width = max((len(r) for r in rows), default=0)
            arr = np.zeros((len(rows), max(width, 2)), dtype=np.int32)
            for i, r in enumerate(rows):
                arr[i, :len(r)] = r
        self.cdfs = arr
        self.sizes = i32(cdf_sizes).reshape(-1)
        self.offsets = i32(offsets).reshape(-1)
        n = arr.shape[0]
        if self.sizes.size != n or self.offsets.size != n:
            raise ValueError("cdfs, cdf_sizes and offsets must have the same length")
        self.struct = RansTables(_ptr(arr), arr.shape[1], _ptr(self.sizes), _ptr(self.offsets), n)

    def ref(self):
        return ctypes.byref(self.struct)


def pmf_to_quantized_cdf_rows(pmf: np.ndarray, lengths: np.ndarray, precision: int, width: int) -> np.ndarray:
    """Row-wise quantized CDFs into a zero-filled [rows, width] int32 table."""
    pmf = np.ascontiguousarray(pmf, dtype=np.float32)
    lengths = i32(lengths)
    rows = lengths.size
    out = np.zeros((rows, width), dtype=np.int32)
    if rows:
        lib.cai_pmf_to_quantized_cdf_rows(_ptr(pmf), pmf.shape[1], _ptr(lengths), rows, int(precision), _ptr(out),
                                          width, default_threads())
    return out


def encode_streams(symbols: np.ndarray, indexes: np.ndarray, tables: Tables, nstreams: int) -> list:
    """Equal-length streams (one per image): symbols/indexes [nstreams, n] -> list of bytes."""
    sym = i32(symbols).reshape(nstreams, -1)
    idx = i32(indexes).reshape(nstreams, -1)
    n = sym.shape[1]
    sym_off = np.arange(nstreams + 1, dtype=np.int64) * n
    cap = int(lib.cai_rans_max_bytes(n))
    out_off = np.arange(nstreams + 1, dtype=np.int64) * cap
    out = np.empty(max(1, nstreams * cap), dtype=np.uint8)
    nbytes = np.zeros(nstreams, dtype=np.int64)
    if nstreams:
        lib.cai_rans_encode_batch(nstreams, _ptr(sym), _ptr(idx), _ptr(sym_off), tables.ref(), _ptr(out),
                                  _ptr(out_off), _ptr(nbytes), default_threads())
    return [out[out_off[s]:out_off[s] + nbytes[s]].tobytes() for s in range(nstreams)]


def decode_streams(strings: Sequence[bytes], indexes: np.ndarray, tables: Tables) -> np.ndarray:
    """Inverse of encode_streams: -> int32 [nstreams, n]."""
    ns = len(strings)
    idx = i32(indexes).reshape(ns, -1)
    n = idx.shape[1]
    blob = np.frombuffer(b"".join(bytes(s) for s in strings) or b"\0", dtype=np.uint8)
    lens = np.array([len(s) for s in strings], dtype=np.int64)
    data_off = np.zeros(ns + 1, dtype=np.int64)
    data_off[1:] = np.cumsum(lens)
    sym_off = np.arange(ns + 1, dtype=np.int64) * n
    out = np.empty((ns, n), dtype=np.int32)
    if ns:
        lib.cai_rans_decode_batch(ns, _ptr(blob), _ptr(data_off), _ptr(lens), _ptr(idx), _ptr(sym_off), tables.ref(),
                                  _ptr(out), default_threads())
    return out
