"""LowerBound (reference: compressai/ops/bound_ops.py:36-80).

On the hot path the bound is applied inside the fused HIP kernels (GDN
reparametrisation, GaussianConditional scale bound, likelihood bound); this
module keeps the ``bound`` buffer (state_dict key ``...lower_bound.bound``)
and offers the op standalone with the same custom gradient:
d/dx max(x, b) passes the gradient iff x >= b or grad < 0.
"""
import torch
import torch.nn as nn


class _LowerBoundFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bound):
        ctx.save_for_backward(x, bound)
        return torch.max(x, bound)

    @staticmethod
    def backward(ctx, g):
        x, bound = ctx.saved_tensors
        return g * ((x >= bound) | (g < 0)).to(g.dtype), None


class LowerBound(nn.Module):
    bound: torch.Tensor

    def __init__(self, bound: float):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def lower_bound(self, x):
        return _LowerBoundFn.apply(x, self.bound.to(x.dtype))

    def forward(self, x):
        return self.lower_bound(x)
