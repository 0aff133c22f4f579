"""L1 ops (reference: compressai/ops/__init__.py:30-34)."""
from .bound_ops import LowerBound
from .parametrizers import NonNegativeParametrizer
from .ops import ste_round

__all__ = ["LowerBound", "NonNegativeParametrizer", "ste_round"]
