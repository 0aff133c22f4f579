"""GDN / IGDN (reference: compressai/layers/gdn.py:38-121) on cai_gdn_* kernels.

Same parameters (``beta``, ``gamma``) and buffers (``beta_reparam.*``,
``gamma_reparam.*``) as the reference; forward = GdnFn (reparametrisation,
x^2 -> C x C MFMA GEMM -> +beta -> rsqrt/sqrt -> *x in one kernel).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import MASK_SIGN
from .._ops import ConvFn, ConvSpec, Gdn1OutFn, GdnFn, compute_dtype
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
        C = x.shape[1]
        cap = 256 if compute_dtype() == torch.bfloat16 else 192
        if C % 32 == 0 and C <= cap:
            return GdnFn.apply(x, self.beta, self.gamma, self.inverse, self.beta_reparam.minimum,
                               self.beta_reparam.reparam_offset)
        # the kernels take channel counts that are multiples of 32 (MFMA K = 32 bf16): pad with zero
        # channels, gamma rows / columns of 0 and beta of 1 -- the real channels' norm is unchanged and the
        # padded outputs (0) are sliced off; autograd routes the gradients back through the padding
        Cp = (C + 31) // 32 * 32
        if Cp > cap:
            raise ValueError(f"GDN: {C} channels; this build supports up to {cap}")
        xp = F.pad(x, (0, 0, 0, 0, 0, Cp - C))
        beta = torch.cat([self.beta, self.beta.new_ones(Cp - C)])
        gamma = F.pad(self.gamma, (0, Cp - C, 0, Cp - C))
        y = GdnFn.apply(xp, beta, gamma, self.inverse, self.beta_reparam.minimum, self.beta_reparam.reparam_offset)
        return y[:, :C]


_GDN1_NORM = ConvSpec(1, 1, 0, in_abs=True, in_mask=MASK_SIGN)


class GDN1(GDN):
    """Simplified GDN (reference gdn.py:95-121): norm = beta + gamma |x|, out = x / norm (inverse: x * norm).

    norm is the 1x1 convolution of |x| on the conv kernels (|x| applied on load, sign(x) on the input
    gradient, gamma / beta reparametrised like the reference), the division is cai_gdn1_out."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        C = x.shape[1]
        beta = self.beta_reparam(self.beta)
        gamma = self.gamma_reparam(self.gamma).reshape(C, C, 1, 1)
        norm = ConvFn.apply(x, gamma, beta, _GDN1_NORM)
        return Gdn1OutFn.apply(x, norm, self.inverse)
