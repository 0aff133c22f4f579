"""NonNegativeParametrizer (reference: compressai/ops/parametrizers.py:38-64).

Holds ``pedestal`` and ``lower_bound.bound``; GDN applies the same map inside
``cai_gdn_reparam`` / ``cai_gdn_param_grad``:
out = max(x, sqrt(minimum + offset^2))^2 - offset^2.
"""
import torch
import torch.nn as nn

from .bound_ops import LowerBound


class NonNegativeParametrizer(nn.Module):
    pedestal: torch.Tensor

    def __init__(self, minimum: float = 0, reparam_offset: float = 2 ** -18):
        super().__init__()
        self.minimum = float(minimum)
        self.reparam_offset = float(reparam_offset)
        self.register_buffer("pedestal", torch.Tensor([self.reparam_offset ** 2]))
        self.lower_bound = LowerBound((self.minimum + self.reparam_offset ** 2) ** 0.5)

    def init(self, x: torch.Tensor) -> torch.Tensor:
        return torch.sqrt(torch.max(x + self.pedestal, self.pedestal))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.lower_bound(x) ** 2 - self.pedestal.to(x.dtype)
