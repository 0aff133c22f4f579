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
from .._ops import ConvFn, ConvSpec


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

    def run(self, x, **kw):
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


class Sequential(nn.Sequential):
    """nn.Sequential with conv+activation epilogue fusion (see module docstring)."""

    def forward(self, x, input_abs: bool = False):
        mods = list(self)
        n = len(mods)
        i = 0
        pending = (MASK_SIGN, 0.0) if input_abs else (MASK_NONE, 0.0)
        first = True
        while i < n:
            m = mods[i]
            if isinstance(m, _CONVS):
                act, prm, skip = ACT_NONE, 0.0, 0
                nxt = mods[i + 1] if i + 1 < n else None
                if isinstance(nxt, nn.ReLU):
                    act, skip = ACT_RELU, 1
                elif isinstance(nxt, nn.LeakyReLU):
                    act, prm, skip = ACT_LEAKY, float(nxt.negative_slope), 1
                after = mods[i + 1 + skip] if i + 1 + skip < n else None
                downstream = act != ACT_NONE and isinstance(after, _CONVS)
                x = m.run(x, act=act, act_param=prm, in_abs=(input_abs and first), in_mask=pending[0],
                          in_mask_param=pending[1], act_bwd_downstream=downstream)
                pending = ((MASK_POS if act == ACT_RELU else MASK_LEAKY), prm) if downstream else (MASK_NONE, 0.0)
                i += 1 + skip
            else:
                if input_abs and first:
                    x = torch.abs(x)
                x = m(x)
                pending = (MASK_NONE, 0.0)
                i += 1
            first = False
        return x
