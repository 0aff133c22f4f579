"""Ballé 2018 / Minnen 2018 models (reference: compressai/models/google.py:58-692).

Same classes, constructor signatures (``channel`` argument of the fork
included), module names and state_dict keys.  Forward passes are the
reference's (google.py:172-182, 281-295, 379-391, 493-515) with two
MI355X-motivated differences that leave the arithmetic unchanged:
  * ``torch.abs(y)`` feeding h_a is applied inside the first h_a conv's
    operand load (and its backward sign mask inside that conv's dgrad);
  * conv -> ReLU/LeakyReLU pairs run fused (layers.Sequential);
and without the reference's debug prints (google.py:287-288).
"""
import math
import warnings

import torch
import torch.nn as nn

from ..entropy_models import EntropyBottleneck, GaussianConditional
from ..layers import GDN, MaskedConv2d, Sequential
from ..layers.conv import Conv2d
from .utils import conv, deconv, update_registered_buffers

__all__ = ["CompressionModel", "FactorizedPrior", "ScaleHyperprior", "MeanScaleHyperprior",
           "JointAutoregressiveHierarchicalPriors", "get_scale_table", "SCALES_MIN", "SCALES_MAX", "SCALES_LEVELS"]

SCALES_MIN = 0.11
SCALES_MAX = 256
SCALES_LEVELS = 64


def get_scale_table(min=SCALES_MIN, max=SCALES_MAX, levels=SCALES_LEVELS):
    return torch.exp(torch.linspace(math.log(min), math.log(max), levels))


class CompressionModel(nn.Module):
    def __init__(self, entropy_bottleneck_channels, init_weights=None):
        super().__init__()
        self.entropy_bottleneck = EntropyBottleneck(entropy_bottleneck_channels)
        if init_weights is not None:
            warnings.warn("init_weights was removed as it was never functional", DeprecationWarning)

    def aux_loss(self):
        return sum(m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck))

    def forward(self, *args):
        raise NotImplementedError()

    def __call__(self, *args, **kwargs):
        # all conv weights are packed to the MFMA layout in one launch per forward
        # (compressai/_prepack.py); the reference has no counterpart (stock convs)
        from .._prepack import prepacked_forward

        with prepacked_forward(self):
            return super().__call__(*args, **kwargs)

    def update(self, force=False):
        updated = False
        for m in self.children():
            if isinstance(m, EntropyBottleneck):
                updated |= m.update(force=force)
        return updated

    def load_state_dict(self, state_dict, strict: bool = True):
        update_registered_buffers(self.entropy_bottleneck, "entropy_bottleneck",
                                  ["_quantized_cdf", "_offset", "_cdf_length"], state_dict)
        return super().load_state_dict(state_dict, strict=strict)


def _analysis(channel, N, M):
    return Sequential(conv(channel, N), GDN(N), conv(N, N), GDN(N), conv(N, N), GDN(N), conv(N, M))


def _synthesis(channel, N, M):
    return Sequential(deconv(M, N), GDN(N, inverse=True), deconv(N, N), GDN(N, inverse=True),
                      deconv(N, N), GDN(N, inverse=True), deconv(N, channel))


class FactorizedPrior(CompressionModel):
    def __init__(self, N, M, channel=3, **kwargs):
        super().__init__(entropy_bottleneck_channels=M, **kwargs)
        self.g_a = _analysis(channel, N, M)
        self.g_s = _synthesis(channel, N, M)
        self.N = N
        self.M = M

    @property
    def downsampling_factor(self) -> int:
        return 2 ** 4

    def forward(self, x):
        y = self.g_a(x)
        y_hat, y_likelihoods = self.entropy_bottleneck(y)
        x_hat = self.g_s(y_hat)
        return {"x_hat": x_hat, "likelihoods": {"y": y_likelihoods}}

    @classmethod
    def from_state_dict(cls, state_dict, channel=3):
        net = cls(state_dict["g_a.0.weight"].size(0), state_dict["g_a.6.weight"].size(0), channel=channel)
        net.load_state_dict(state_dict)
        return net


class ScaleHyperprior(CompressionModel):
    def __init__(self, N, M, channel=3, **kwargs):
        super().__init__(entropy_bottleneck_channels=N, **kwargs)
        self.g_a = _analysis(channel, N, M)
        self.g_s = _synthesis(channel, N, M)
        self.h_a = Sequential(conv(M, N, stride=1, kernel_size=3), nn.ReLU(inplace=True),
                              conv(N, N), nn.ReLU(inplace=True), conv(N, N))
        self.h_s = Sequential(deconv(N, N), nn.ReLU(inplace=True), deconv(N, N), nn.ReLU(inplace=True),
                              conv(N, M, stride=1, kernel_size=3), nn.ReLU(inplace=True))
        self.gaussian_conditional = GaussianConditional(None)
        self.N = int(N)
        self.M = int(M)

    @property
    def downsampling_factor(self) -> int:
        return 2 ** (4 + 2)

    def forward(self, x):
        y = self.g_a(x)
        z = self.h_a(y, input_abs=True)          # h_a(|y|)
        z_hat, z_likelihoods = self.entropy_bottleneck(z)
        scales_hat = self.h_s(z_hat)
        y_hat, y_likelihoods = self.gaussian_conditional(y, scales_hat)
        x_hat = self.g_s(y_hat)
        return {"x_hat": x_hat, "likelihoods": {"y": y_likelihoods, "z": z_likelihoods}}

    def load_state_dict(self, state_dict, strict: bool = True):
        update_registered_buffers(self.gaussian_conditional, "gaussian_conditional",
                                  ["_quantized_cdf", "_offset", "_cdf_length", "scale_table"], state_dict)
        return super().load_state_dict(state_dict, strict=strict)

    @classmethod
    def from_state_dict(cls, state_dict, channel=3):
        net = cls(state_dict["g_a.0.weight"].size(0), state_dict["g_a.6.weight"].size(0), channel=channel)
        net.load_state_dict(state_dict)
        return net

    def update(self, scale_table=None, force=False):
        if scale_table is None:
            scale_table = get_scale_table()
        updated = self.gaussian_conditional.update_scale_table(scale_table, force=force)
        updated |= super().update(force=force)
        return updated


class MeanScaleHyperprior(ScaleHyperprior):
    def __init__(self, N, M, channel=3, **kwargs):
        super().__init__(N, M, channel, **kwargs)
        self.h_a = Sequential(conv(M, N, stride=1, kernel_size=3), nn.LeakyReLU(inplace=True),
                              conv(N, N), nn.LeakyReLU(inplace=True), conv(N, N))
        self.h_s = Sequential(deconv(N, M), nn.LeakyReLU(inplace=True), deconv(M, M * 3 // 2),
                              nn.LeakyReLU(inplace=True), conv(M * 3 // 2, M * 2, stride=1, kernel_size=3))

    def forward(self, x):
        y = self.g_a(x)
        z = self.h_a(y)
        z_hat, z_likelihoods = self.entropy_bottleneck(z)
        scales_hat, means_hat = self.h_s(z_hat).chunk(2, 1)
        y_hat, y_likelihoods = self.gaussian_conditional(y, scales_hat, means=means_hat)
        x_hat = self.g_s(y_hat)
        return {"x_hat": x_hat, "likelihoods": {"y": y_likelihoods, "z": z_likelihoods}}


class JointAutoregressiveHierarchicalPriors(MeanScaleHyperprior):
    def __init__(self, N=192, M=192, channel=3, **kwargs):
        super().__init__(N=N, M=M, channel=channel, **kwargs)
        self.entropy_parameters = Sequential(
            Conv2d(M * 12 // 3, M * 10 // 3, 1), nn.LeakyReLU(inplace=True),
            Conv2d(M * 10 // 3, M * 8 // 3, 1), nn.LeakyReLU(inplace=True),
            Conv2d(M * 8 // 3, M * 6 // 3, 1))
        self.context_prediction = MaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)

    def forward(self, x):
        y = self.g_a(x)
        z = self.h_a(y)
        z_hat, z_likelihoods = self.entropy_bottleneck(z)
        params = self.h_s(z_hat)
        y_hat = self.gaussian_conditional.quantize(y, "noise" if self.training else "dequantize")
        ctx_params = self.context_prediction(y_hat)
        gaussian_params = self.entropy_parameters(torch.cat((params, ctx_params), dim=1))
        scales_hat, means_hat = gaussian_params.chunk(2, 1)
        _, y_likelihoods = self.gaussian_conditional(y, scales_hat, means=means_hat)
        x_hat = self.g_s(y_hat)
        return {"x_hat": x_hat, "likelihoods": {"y": y_likelihoods, "z": z_likelihoods}}
