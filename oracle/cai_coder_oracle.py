"""CPU oracle for the entropy-coding side (quantized CDFs + rANS bitstreams).

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` as the checker of
``libcai_coder.so``; nothing in the product package imports it.

A pure-Python restatement, for small inputs, of
  * ``pmf_to_quantized_cdf``  -- compressai/cpp_exts/ops/ops.cpp:40-109
  * the rANS coder            -- compressai/cpp_exts/rans/rans_interface.cpp:48-359
    over the 64-bit-state primitives of third_party/ryg_rans/rans64.h:59-142
(paths under /root/reference/CompressAI).  Python integers are exact, so the
only float step -- ``std::round(p * (1 << precision))`` on a C ``float`` --
is done in numpy float32.

Pinning: the reference's only known answer for this code is
``pmf_to_quantized_cdf([0.1, 0.2, 0, 0], 16) == [0, 21845, 65534, 65535,
65536]`` (tests/test_ops.py:103-106), checked in tests/test_coder.py.  The
rANS byte streams are pinned by this restatement alone (the reference may
not be run here) plus the round-trip property the reference's
own tests assert (tests/test_entropy_models.py:258-283): "parity pinned by
one KAT + round trips; stream bytes restatement-defined".
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

PRECISION = 16          # rans_interface.cpp:49
BYPASS_PRECISION = 4    # rans_interface.cpp:51
MAX_BYPASS_VAL = (1 << BYPASS_PRECISION) - 1
RANS64_L = 1 << 31      # rans64.h:59
MASK32 = (1 << 32) - 1


def pmf_to_quantized_cdf(pmf: Sequence[float], precision: int = 16) -> List[int]:
    """ops.cpp:40-109 (pmf elements are C floats: the pybind layer converts to std::vector<float>)."""
    p32 = np.asarray(pmf, dtype=np.float32)
    for p in p32:
        if p < 0 or not np.isfinite(p):
            raise ValueError(f"Invalid `pmf`, non-finite or negative element found: {p}")
    scaled = p32 * np.float32(1 << precision)                           # float * int -> float
    # std::round: half away from zero
    rounded = np.where(scaled >= 0, np.floor(scaled + np.float32(0.5)), np.ceil(scaled - np.float32(0.5)))
    cdf = [0] + [int(v) & MASK32 for v in rounded]
    total = sum(cdf) & MASK32                                           # std::accumulate(.., 0)
    if total == 0:
        raise ValueError("Invalid `pmf`: at least one element must have a non-zero probability.")
    cdf = [((1 << precision) * v // total) & MASK32 for v in cdf]
    for i in range(1, len(cdf)):                                        # std::partial_sum (uint32)
        cdf[i] = (cdf[i] + cdf[i - 1]) & MASK32
    cdf[-1] = 1 << precision
    for i in range(len(cdf) - 1):                                       # :74-100 frequency stealing
        if cdf[i] == cdf[i + 1]:
            best_freq, best_steal = MASK32, -1
            for j in range(len(cdf) - 1):
                freq = (cdf[j + 1] - cdf[j]) & MASK32
                if 1 < freq < best_freq:
                    best_freq, best_steal = freq, j
            if best_steal < 0:
                raise ValueError("no frequency to steal")
            if best_steal < i:
                for j in range(best_steal + 1, i + 1):
                    cdf[j] -= 1
            else:
                for j in range(i + 1, best_steal + 1):
                    cdf[j] += 1
    return cdf


def _symbols(symbols, indexes, cdfs, cdf_sizes, offsets):
    """rans_interface.cpp:117-172: (start, range, bypass) list."""
    out = []
    for sym, idx in zip(symbols, indexes):
        cdf = cdfs[idx]
        max_value = cdf_sizes[idx] - 2
        value = sym - offsets[idx]
        raw_val = 0
        if value < 0:
            raw_val = -2 * value - 1
            value = max_value
        elif value >= max_value:
            raw_val = 2 * (value - max_value)
            value = max_value
        out.append((cdf[value] & 0xFFFF, (cdf[value + 1] - cdf[value]) & 0xFFFF, False))
        if value == max_value:
            n_bypass = 0
            while (raw_val >> (n_bypass * BYPASS_PRECISION)) != 0:
                n_bypass += 1
            val = n_bypass
            while val >= MAX_BYPASS_VAL:
                out.append((MAX_BYPASS_VAL, MAX_BYPASS_VAL + 1, True))
                val -= MAX_BYPASS_VAL
            out.append((val, val + 1, True))
            for j in range(n_bypass):
                v = (raw_val >> (j * BYPASS_PRECISION)) & MAX_BYPASS_VAL
                out.append((v, v + 1, True))
    return out


def _flush(syms) -> bytes:
    """rans_interface.cpp:175-200 with Rans64EncPut / PutBits / Flush (rans64.h:77-103)."""
    x = RANS64_L
    words: List[int] = []     # emitted in reverse order (the reference writes backwards)
    for start, rng, bypass in reversed(syms):
        if not bypass:
            x_max = ((RANS64_L >> PRECISION) << 32) * rng
            if x >= x_max:
                words.append(x & MASK32)
                x >>= 32
            x = ((x // rng) << PRECISION) + (x % rng) + start
        else:
            x_max = ((RANS64_L >> 16) << 32) * (1 << (16 - BYPASS_PRECISION))
            if x >= x_max:
                words.append(x & MASK32)
                x >>= 32
            x = (x << BYPASS_PRECISION) | start
    stream = [x & MASK32, (x >> 32) & MASK32] + list(reversed(words))
    return b"".join(int(w).to_bytes(4, "little") for w in stream)


def encode_with_indexes(symbols, indexes, cdfs, cdf_sizes, offsets) -> bytes:
    """RansEncoder.encode_with_indexes (rans_interface.cpp:202-213)."""
    return _flush(_symbols(symbols, indexes, cdfs, cdf_sizes, offsets))


class BufferedRansEncoder:
    """rans_interface.cpp:108-200."""

    def __init__(self):
        self._syms = []

    def encode_with_indexes(self, symbols, indexes, cdfs, cdf_sizes, offsets):
        self._syms.extend(_symbols(symbols, indexes, cdfs, cdf_sizes, offsets))

    def flush(self) -> bytes:
        s, self._syms = _flush(self._syms), []
        return s


class _Dec:
    def __init__(self, data: bytes):
        self.w = [int.from_bytes(data[i:i + 4], "little") for i in range(0, len(data) - len(data) % 4, 4)]
        self.x = self.w[0] | (self.w[1] << 32)
        self.p = 2

    def _renorm(self):
        if self.x < RANS64_L:
            self.x = (self.x << 32) | self.w[self.p]
            self.p += 1

    def get_bits(self, n):                       # rans_interface.cpp:89-105
        v = self.x & ((1 << n) - 1)
        self.x >>= n
        self._renorm()
        return v

    def symbol(self, idx, cdfs, cdf_sizes, offsets):   # rans_interface.cpp:231-281
        cdf = cdfs[idx]
        max_value = cdf_sizes[idx] - 2
        cum = self.x & ((1 << PRECISION) - 1)
        s = next(j for j in range(cdf_sizes[idx]) if cdf[j] > cum) - 1
        self.x = (cdf[s + 1] - cdf[s]) * (self.x >> PRECISION) + (self.x & ((1 << PRECISION) - 1)) - cdf[s]
        self._renorm()
        value = s
        if value == max_value:
            val = self.get_bits(BYPASS_PRECISION)
            n_bypass = val
            while val == MAX_BYPASS_VAL:
                val = self.get_bits(BYPASS_PRECISION)
                n_bypass += val
            raw_val = 0
            for j in range(n_bypass):
                raw_val |= self.get_bits(BYPASS_PRECISION) << (j * BYPASS_PRECISION)
            value = raw_val >> 1
            value = -value - 1 if raw_val & 1 else value + max_value
        return value + offsets[idx]


def decode_with_indexes(data: bytes, indexes, cdfs, cdf_sizes, offsets) -> List[int]:
    """RansDecoder.decode_with_indexes (rans_interface.cpp:215-284)."""
    d = _Dec(data)
    return [d.symbol(i, cdfs, cdf_sizes, offsets) for i in indexes]
