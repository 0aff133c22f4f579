"""Layer zoo (reference: compressai/layers/layers.py:40-244).

MaskedConv2d follows layers.py:52-78: the weight is masked in place before
every call (so gradients reach masked taps exactly as in the reference), then
the conv runs on the HIP implicit-GEMM kernel.

The residual / attention blocks of the cheng2020 models (layers.py:97-244)
keep the reference's module tree (so state_dict keys match: ``conv1``,
``conv2``, ``gdn``, ``skip``, ``subpel_conv.0``, ``upsample.0``,
``conv_a.0.conv.2`` ...).  Their forward passes chain the HIP convs with the
activation in the conv epilogue and its backward mask in the next conv's
dgrad epilogue.  ResidualUnit's ``+ x`` and trailing ReLU run in its last
conv's epilogue (cai_conv_fwd_res); the other residual adds, the attention
gate and the pixel shuffle run on the elementwise kernels
(csrc/elementwise.hip).
"""
import os
from typing import Any

import torch
import torch.nn as nn

from .._native import ACT_LEAKY, ACT_NONE, ACT_RELU, MASK_LEAKY, MASK_POS
from .._ops import (AddActFn, AttentionBlockFn, GateFn, ResidualBlockFn, ResidualChainFn, _ab_side, fan_out,
                    residual_fusable)
from .conv import Conv2d, ConvTranspose2d, PixelShuffle, Sequential
from .gdn import GDN

__all__ = ["MaskedConv2d", "conv1x1", "conv3x3", "subpel_conv3x3", "PixelShuffle", "ResidualBlockWithStride",
           "ResidualBlockUpsample", "ResidualBlock", "AttentionBlock"]

_SLOPE = 0.01   # nn.LeakyReLU() default negative_slope


class MaskedConv2d(Conv2d):
    def __init__(self, *args: Any, mask_type: str = "A", **kwargs: Any):
        super().__init__(*args, **kwargs)
        if mask_type not in ("A", "B"):
            raise ValueError(f'Invalid "mask_type" value "{mask_type}"')
        self.register_buffer("mask", torch.ones_like(self.weight.data))
        _, _, h, w = self.mask.size()
        self.mask[:, :, h // 2, w // 2 + (mask_type == "B"):] = 0
        self.mask[:, :, h // 2 + 1:] = 0

    def run(self, x, **kw):
        self.weight.data *= self.mask
        return super().run(x, **kw)


def conv3x3(in_ch: int, out_ch: int, stride: int = 1) -> nn.Module:
    return Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def conv1x1(in_ch: int, out_ch: int, stride: int = 1) -> nn.Module:
    return Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


def subpel_conv3x3(in_ch: int, out_ch: int, r: int = 1) -> nn.Module:
    """layers.py:86-91: conv3x3 to out_ch*r^2 channels, then PixelShuffle(r)."""
    return Sequential(Conv2d(in_ch, out_ch * r ** 2, kernel_size=3, padding=1), PixelShuffle(r))


def _join(main, side, x, identity):
    """The side branch joins the caller's stream; caching-allocator bookkeeping of the tensors that crossed."""
    main.wait_stream(side)
    x.record_stream(side)
    identity.record_stream(main)


class ResidualBlockWithStride(nn.Module):
    """layers.py:97-129: conv3x3(s) -> LeakyReLU -> conv3x3 -> GDN, + skip (conv1x1(s) or identity)."""

    def __init__(self, in_ch: int, out_ch: int, stride: int = 2):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch, stride=stride)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(out_ch, out_ch)
        self.gdn = GDN(out_ch)
        self.skip = conv1x1(in_ch, out_ch, stride=stride) if (stride != 1 or in_ch != out_ch) else None

    def forward(self, x):
        side = _ab_side(x, self.skip.parameters()) if self.skip is not None else None
        xm, xs = fan_out(x, absorb=False)   # x's two gradients: one native add, not autograd's ATen add
        if side is not None:   # the skip conv on the side stream (autograd runs its backward there too)
            main = torch.cuda.current_stream(x.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                identity = self.skip(xs)
        out = self.conv1.run(xm, act=ACT_LEAKY, act_param=_SLOPE, act_bwd_downstream=True)
        out = self.conv2.run(out, in_mask=MASK_LEAKY, in_mask_param=_SLOPE)
        out = self.gdn(out)
        if side is not None:
            _join(main, side, x, identity)
        else:
            identity = self.skip(xs) if self.skip is not None else xs
        return AddActFn.apply(out, identity, ACT_NONE, 0.0)


class ResidualBlockUpsample(nn.Module):
    """layers.py:132-159: subpel_conv3x3 -> LeakyReLU -> conv3x3 -> IGDN, + subpel_conv3x3(x)."""

    def __init__(self, in_ch: int, out_ch: int, upsample: int = 2):
        super().__init__()
        self.subpel_conv = subpel_conv3x3(in_ch, out_ch, upsample)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv = conv3x3(out_ch, out_ch)
        self.igdn = GDN(out_ch, inverse=True)
        self.upsample = subpel_conv3x3(in_ch, out_ch, upsample)

    def forward(self, x):
        side = _ab_side(x, self.upsample.parameters())
        xm, xu = fan_out(x, absorb=False)
        if side is not None:   # the upsampling branch on the side stream (autograd runs its backward there too)
            main = torch.cuda.current_stream(x.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                identity = self.upsample(xu)
        out = self.subpel_conv(xm, act=ACT_LEAKY, act_param=_SLOPE, act_bwd_downstream=True)
        out = self.conv.run(out, in_mask=MASK_LEAKY, in_mask_param=_SLOPE)
        out = self.igdn(out)
        if side is not None:
            _join(main, side, x, identity)
        else:
            identity = self.upsample(xu)
        return AddActFn.apply(out, identity, ACT_NONE, 0.0)


class ResidualBlock(nn.Module):
    """layers.py:162-193: conv3x3 -> LeakyReLU -> conv3x3 -> LeakyReLU, + skip (conv1x1 or identity)."""

    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(out_ch, out_ch)
        self.skip = conv1x1(in_ch, out_ch) if in_ch != out_ch else None

    # False: the per-module chain (autograd sums x's two gradients); CAI_RESIDUAL_FUSE=0 for A/Bs
    fuse_residual = os.environ.get("CAI_RESIDUAL_FUSE", "1") != "0"

    def forward(self, x):
        s1 = self.conv1._spec(act=ACT_LEAKY, act_param=_SLOPE, act_bwd_downstream=True)
        s2 = self.conv2._spec(act=ACT_LEAKY, act_param=_SLOPE, in_mask=MASK_LEAKY, in_mask_param=_SLOPE)
        if self.skip is None and self.fuse_residual:
            return ResidualBlockFn.apply(x, s1, s2, self.conv1.weight, self.conv1.bias, self.conv2.weight,
                                         self.conv2.bias)
        xm, xs = fan_out(x, absorb=False)
        out = self.conv1.run(xm, act=ACT_LEAKY, act_param=_SLOPE, act_bwd_downstream=True)
        out = self.conv2.run(out, act=ACT_LEAKY, act_param=_SLOPE, in_mask=MASK_LEAKY, in_mask_param=_SLOPE)
        identity = self.skip(xs) if self.skip is not None else xs
        return AddActFn.apply(out, identity, ACT_NONE, 0.0)


class ResidualUnit(nn.Module):
    """AttentionBlock's inner unit (layers.py:211-226): relu(conv1x1 -> ReLU -> conv3x3 -> ReLU -> conv1x1 + x)."""

    def __init__(self, N: int):
        super().__init__()
        self.conv = Sequential(conv1x1(N, N // 2), nn.ReLU(inplace=True), conv3x3(N // 2, N // 2),
                               nn.ReLU(inplace=True), conv1x1(N // 2, N))
        self.relu = nn.ReLU(inplace=True)

    # False: the unfused chain (Sequential, then add + ReLU on the elementwise kernel); CAI_RESIDUAL_FUSE=0 for A/Bs
    fuse_residual = os.environ.get("CAI_RESIDUAL_FUSE", "1") != "0"

    def fusable(self) -> bool:
        return self.fuse_residual and residual_fusable(self.conv[4]._spec(act=ACT_RELU, in_mask=MASK_POS))

    def chain_args(self):
        """(specs, params) of this unit in ResidualChainFn: the Sequential's fusion, with `+ x` and the trailing
        ReLU in the last conv's epilogue."""
        c = self.conv
        specs = (c[0]._spec(act=ACT_RELU, act_bwd_downstream=True),
                 c[2]._spec(act=ACT_RELU, in_mask=MASK_POS, act_bwd_downstream=True),
                 c[4]._spec(act=ACT_RELU, in_mask=MASK_POS))
        return specs, (c[0].weight, c[0].bias, c[2].weight, c[2].bias, c[4].weight, c[4].bias)

    def forward(self, x):
        if not self.fusable():
            return AddActFn.apply(self.conv(x), x, ACT_RELU, 0.0)
        return residual_chain([self], x)


def chain_fusable(units) -> bool:
    return all(u.fusable() for u in units)


def residual_chain(units, x, out_masked: bool = False):
    """ResidualUnits applied in sequence, as one ResidualChainFn node (fusable units only).  out_masked: the
    caller's consumer applies the last unit's ReLU mask to the gradient (MASK_POS dgrad, GateFn relu_a)."""
    specs, params = _chain_specs(units)
    return ResidualChainFn.apply(x, specs, bool(out_masked), *params)


def _chain_specs(units):
    specs, params = [], []
    for u in units:
        sp, pr = u.chain_args()
        specs.append(sp)
        params.extend(pr)
    return tuple(specs), params


class AttentionBlock(nn.Module):
    """layers.py:196-244: x + conv_a(x) * sigmoid(conv_b(x))."""

    def __init__(self, N: int):
        super().__init__()
        self.conv_a = Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N))
        self.conv_b = Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N), conv1x1(N, N))

    def forward(self, x):
        ua, ub = list(self.conv_a), list(self.conv_b)[:3]
        if not (chain_fusable(ua) and chain_fusable(ub)):
            return GateFn.apply(self.conv_a(x), self.conv_b(x), x)
        # one autograd node: each branch's three ResidualUnits as a chain (layers.py:225-236), the chains' last
        # ReLU masks in their consumers' backward (conv_b's 1x1 conv dgrad MASK_POS, the gate's da), x's three
        # gradients summed in the branches' first dgrad epilogues
        sa, pa = _chain_specs(ua)
        sb, pb = _chain_specs(ub)
        c3 = self.conv_b[3]
        return AttentionBlockFn.apply(x, sa, sb, c3._spec(in_mask=MASK_POS), *pa, *pb, c3.weight, c3.bias)
