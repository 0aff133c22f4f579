"""``compressai.ans`` (reference: cpp_exts/rans/rans_interface.cpp:361-381), backed by libcai_coder.so.

Same classes, methods and argument types (python lists of ints, ``bytes``
streams); the streams are byte-identical to the reference coder's.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from ._coder import Tables, _ptr, i32, lib

__all__ = ["RansEncoder", "BufferedRansEncoder", "RansDecoder"]


class RansEncoder:
    def encode_with_indexes(self, symbols: Sequence[int], indexes: Sequence[int], cdfs, cdfs_sizes: Sequence[int],
                            offsets: Sequence[int]) -> bytes:
        t = Tables(cdfs, cdfs_sizes, offsets)
        sym, idx = i32(symbols).reshape(-1), i32(indexes).reshape(-1)
        if sym.size != idx.size:
            raise ValueError("symbols and indexes must have the same length")
        cap = int(lib.cai_rans_max_bytes(sym.size))
        out = np.empty(max(cap, 8), dtype=np.uint8)
        nbytes = np.zeros(1, dtype=np.int64)
        lib.cai_rans_encode(_ptr(sym), _ptr(idx), sym.size, t.ref(), _ptr(out), out.size, _ptr(nbytes))
        return out[:int(nbytes[0])].tobytes()


class BufferedRansEncoder:
    def __init__(self):
        self._h = lib.cai_rans_buffered_create()
        if not self._h:
            raise MemoryError("cai_rans_buffered_create failed")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            lib.cai_rans_buffered_destroy(h)

    def encode_with_indexes(self, symbols, indexes, cdfs, cdfs_sizes, offsets) -> None:
        t = Tables(cdfs, cdfs_sizes, offsets)
        sym, idx = i32(symbols).reshape(-1), i32(indexes).reshape(-1)
        if sym.size != idx.size:
            raise ValueError("symbols and indexes must have the same length")
        lib.cai_rans_buffered_encode(self._h, _ptr(sym), _ptr(idx), sym.size, t.ref())

    def flush(self) -> bytes:
        cap = int(lib.cai_rans_buffered_max_bytes(self._h))
        out = np.empty(max(cap, 8), dtype=np.uint8)
        nbytes = np.zeros(1, dtype=np.int64)
        lib.cai_rans_buffered_flush(self._h, _ptr(out), out.size, _ptr(nbytes))
        return out[:int(nbytes[0])].tobytes()


class RansDecoder:
    def __init__(self):
        self._h = lib.cai_rans_decoder_create()
        if not self._h:
            raise MemoryError("cai_rans_decoder_create failed")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            lib.cai_rans_decoder_destroy(h)

    def decode_with_indexes(self, encoded: bytes, indexes, cdfs, cdfs_sizes, offsets) -> List[int]:
        t = Tables(cdfs, cdfs_sizes, offsets)
        idx = i32(indexes).reshape(-1)
        data = np.frombuffer(bytes(encoded) or b"\0", dtype=np.uint8)
        out = np.empty(idx.size, dtype=np.int32)
        lib.cai_rans_decode(_ptr(data), len(encoded), _ptr(idx), idx.size, t.ref(), _ptr(out))
        return out.tolist()

    def set_stream(self, encoded: bytes) -> None:
        data = np.frombuffer(bytes(encoded) or b"\0", dtype=np.uint8)
        lib.cai_rans_decoder_set_stream(self._h, _ptr(data), len(encoded))

    def decode_stream(self, indexes, cdfs, cdfs_sizes, offsets) -> List[int]:
        t = Tables(cdfs, cdfs_sizes, offsets)
        idx = i32(indexes).reshape(-1)
        out = np.empty(idx.size, dtype=np.int32)
        lib.cai_rans_decoder_decode_stream(self._h, _ptr(idx), idx.size, t.ref(), _ptr(out))
        return out.tolist()
