"""Conv2d / ConvTranspose2d on the libcai implicit-GEMM kernels.

Drop-in subclasses of torch.nn.Conv2d / ConvTranspose2d: same constructor,
parameters (``weight``, ``bias``), default init and state_dict keys, so
checkpoints interchange with the reference (models/utils.py:128-146 builds
them).  ``forward`` runs ConvFn (cai_conv_fwd / _dgrad / _wgrad).

``Sequential`` fuses ``conv -> ReLU/LeakyReLU`` pairs: the activation runs in
the conv epilogue, and when the activated tensor feeds the next conv its
backward mask is applied in that conv's dgrad epilogue (MASK_POS/LEAKY) -- no
separate elementwise kernels.  Indices (and so state_dict keys such as
``h_a.2.weight``) are those of the reference Sequentials.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .._native import ACT_LEAKY, ACT_NONE, ACT_RELU, MASK_LEAKY, MASK_NONE, MASK_POS, MASK_SIGN
from .._ops import ActFn, ConvFn, ConvSpec, PixelShuffleFn


def _square(v, name):
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            raise ValueError(f"{name} must be square/symmetric on the MI355X path, got {v}")
        return int(v[0])
    return int(v)


class _ConvMixin:
    def _spec(self, act=ACT_NONE, act_param=0.0, in_abs=False, in_mask=MASK_NONE, in_mask_param=0.0,
              act_bwd_downstream=False, out_channels=None):
        if self.groups != 1 or _square(self.dilation, "dilation") != 1:
            raise ValueError("groups/dilation other than 1 are not supported")
        if self.padding_mode != "zeros":
            raise ValueError("only zero padding is supported")
        transposed = isinstance(self, nn.ConvTranspose2d)
        op = _square(self.output_padding, "output_padding") if transposed else 0
        cout = self.out_channels if out_channels is None else out_channels
        return ConvSpec(_square(self.kernel_size, "kernel_size"), _square(self.stride, "stride"),
                        _square(self.padding, "padding"), op, transposed, act, act_param, in_abs,
                        out_nchw32=(cout % 8 != 0), in_mask=in_mask, in_mask_param=in_mask_param,
                        act_bwd_downstream=act_bwd_downstream)

    def run(self, x, res=None, **kw):
        if res is not None:   # y = act(conv(x) + bias + res) in the epilogue (ResidualUnit)
            return ConvFn.apply(x, self.weight, self.bias, self._spec(**kw), res)
        return ConvFn.apply(x, self.weight, self.bias, self._spec(**kw))


class Conv2d(_ConvMixin, nn.Conv2d):
    def forward(self, x):
        return self.run(x)


class ConvTranspose2d(_ConvMixin, nn.ConvTranspose2d):
    def forward(self, x, output_size=None):
        if output_size is not None:
            raise ValueError("output_size is not supported; use output_padding")
        return self.run(x)


_CONVS = (Conv2d, ConvTranspose2d)


def _act_of(m):
    if isinstance(m, nn.ReLU):
        return ACT_RELU, 0.0
    if isinstance(m, nn.LeakyReLU):
        return ACT_LEAKY, float(m.negative_slope)
    return ACT_NONE, 0.0


class PixelShuffle(nn.PixelShuffle):
    """nn.PixelShuffle on the HIP permutation kernel (pixel-major in -> pixel-major out)."""

    def forward(self, x):
        return PixelShuffleFn.apply(x, int(self.upscale_factor))


def _is_subpel(m):
    """Sequential(conv, PixelShuffle) as built by subpel_conv3x3 (layers.py:86-91)."""
    return (isinstance(m, Sequential) and len(m) == 2 and isinstance(m[0], _CONVS)
            and isinstance(m[1], nn.PixelShuffle))


class Sequential(nn.Sequential):
    """nn.Sequential with conv+activation epilogue fusion (see module docstring).

    A sub-pixel block (conv, PixelShuffle) counts as a conv: an activation after
    it runs in the conv epilogue (the permutation commutes with it), and its
    backward mask in the next conv's dgrad epilogue, whose aux input is the
    shuffled activation.  ``act`` applies a trailing activation requested by an
    enclosing Sequential."""

    def forward(self, x, input_abs: bool = False, act: int = ACT_NONE, act_param: float = 0.0,
                in_mask: int = MASK_NONE, in_mask_param: float = 0.0, act_bwd_downstream: bool = False):
        mods = list(self)
        n = len(mods)
        i = 0
        pending = (MASK_SIGN, 0.0) if input_abs else (in_mask, in_mask_param)
        first = True
        cuts = self.__dict__.get("_cut_fns")
        while i < n:
            m = mods[i]
            if cuts and i in cuts:
                # a gradient-bucket cut at this child's input (compressai.distributed): children are called
                # through .run(), which bypasses forward pre-hooks
                x = cuts[i](x)
            convlike = isinstance(m, _CONVS) or _is_subpel(m)
            if convlike:
                a, prm = _act_of(mods[i + 1]) if i + 1 < n else (ACT_NONE, 0.0)
                skip = 1 if a != ACT_NONE else 0
                # last producer: only permutations (PixelShuffle) follow it
                last = all(isinstance(mm, nn.PixelShuffle) for mm in mods[i + 1 + skip:])
                if last and a == ACT_NONE and act != ACT_NONE:
                    a, prm = act, act_param           # the enclosing Sequential's activation
                after = mods[i + 1 + skip] if i + 1 + skip < n else None
                if last:
                    downstream = a != ACT_NONE and act_bwd_downstream
                else:
                    downstream = a != ACT_NONE and (isinstance(after, _CONVS) or _is_subpel(after))
                kw = dict(act=a, act_param=prm, in_mask=pending[0], in_mask_param=pending[1],
                          act_bwd_downstream=downstream)
                if isinstance(m, _CONVS):
                    x = m.run(x, in_abs=(input_abs and first), **kw)
                else:
                    x = m(x, input_abs=(input_abs and first), **kw)
                pending = ((MASK_POS if a == ACT_RELU else MASK_LEAKY), prm) if downstream else (MASK_NONE, 0.0)
                i += 1 + skip
            else:
                if input_abs and first:
                    x = torch.abs(x)
                a, prm = _act_of(m)
                x = ActFn.apply(x, a, prm) if a != ACT_NONE else m(x)
                pending = (MASK_NONE, 0.0)
                i += 1
            first = False
        if cuts:
            # every cut must fall on a child this loop starts (not inside a fused conv + activation pair)
            visited = set()
            j = 0
            while j < n:
                visited.add(j)
                mm = mods[j]
                fused = (isinstance(mm, _CONVS) or _is_subpel(mm)) and j + 1 < n and _act_of(mods[j + 1])[0] != ACT_NONE
                j += 2 if fused else 1
            bad = [c for c in cuts if c not in visited]
            if bad:
                raise ValueError(f"Sequential: gradient-bucket cut at child {bad} falls inside a fused conv + activation")
        if act != ACT_NONE and not (n and (isinstance(mods[-1], _CONVS) or _is_subpel(mods[-1])
                                           or isinstance(mods[-1], nn.PixelShuffle))):
            x = ActFn.apply(x, act, act_param)
        return x
