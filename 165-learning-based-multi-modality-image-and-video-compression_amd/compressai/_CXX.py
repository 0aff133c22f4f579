"""``compressai._CXX`` (reference: cpp_exts/ops/ops.cpp:111-118), backed by libcai_coder.so."""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from ._coder import _ptr, lib

__all__ = ["pmf_to_quantized_cdf"]


def pmf_to_quantized_cdf(pmf: Sequence[float], precision: int) -> List[int]:
    """Quantized CDF (len(pmf) + 1 entries) of a pmf (ops.cpp:40-109); ValueError on a negative,
    non-finite or all-zero pmf, like the reference's std::domain_error."""
    p = np.ascontiguousarray(np.asarray(pmf, dtype=np.float32).reshape(-1))
    if p.size == 0:
        raise ValueError("Invalid `pmf`: at least one element must have a non-zero probability.")
    out = np.empty(p.size + 1, dtype=np.int32)
    lib.cai_pmf_to_quantized_cdf(_ptr(p), p.size, int(precision), _ptr(out))
    return out.tolist()
