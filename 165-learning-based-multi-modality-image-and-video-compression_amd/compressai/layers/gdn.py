"""GDN / IGDN (reference: compressai/layers/gdn.py:38-121) on cai_gdn_* kernels.

Same parameters (``beta``, ``gamma``) and buffers (``beta_reparam.*``,
``gamma_reparam.*``) as the reference; forward = GdnFn (reparametrisation,
x^2 -> C x C MFMA GEMM -> +beta -> rsqrt/sqrt -> *x in one kernel).
"""
import torch
import torch.nn as nn

from .._ops import GdnFn
from ..ops.parametrizers import NonNegativeParametrizer

__all__ = ["GDN", "GDN1"]


class GDN(nn.Module):
    def __init__(self, in_channels: int, inverse: bool = False, beta_min: float = 1e-6, gamma_init: float = 0.1):
        super().__init__()
        self.inverse = bool(inverse)
        self.beta_reparam = NonNegativeParametrizer(minimum=float(beta_min))
        self.beta = nn.Parameter(self.beta_reparam.init(torch.ones(in_channels)))
        self.gamma_reparam = NonNegativeParametrizer()
        self.gamma = nn.Parameter(self.gamma_reparam.init(float(gamma_init) * torch.eye(in_channels)))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return GdnFn.apply(x, self.beta, self.gamma, self.inverse, self.beta_reparam.minimum,
                           self.beta_reparam.reparam_offset)


class GDN1(GDN):
    """Simplified GDN (|x| instead of x^2, 1/norm instead of rsqrt) -- not used by any benchmarked model."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError("GDN1 is not on the MI355X hot path (no reference config uses it)")
