"""CPU oracle for the learned-compression RD-training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this module;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use it, and only as the checker / the timed CPU baseline.

What it is
----------
An op-for-op fp32 restatement, on CPU PyTorch, of the reference's hot path
(``/root/reference/CompressAI``; every function cites the file:line it
follows).  The reference's forward/backward is itself a composition of stock
torch ops, so running the same composition on this image's torch CPU build
reproduces its arithmetic (up to torch-version drift).

Pinning
-------
The reference may not be imported or executed here.
This oracle is pinned by the reference's own known-answer tests, transcribed
in ``tests/test_oracle_kats.py``:
  * GDN / IGDN closed forms at init (tests/test_layers.py:134-172)
  * quantize semantics (tests/test_entropy_models.py:54-99,177-221,326-363)
  * LowerBound value + gradient rule (tests/test_ops.py:50-73)
  * NonNegativeParametrizer (tests/test_ops.py:75-101)
  * model output keys / likelihood shapes (tests/test_models.py:77-181)
  * CompressionModel parameter count (tests/test_models.py:53-58)
  * scale table endpoints (tests/test_models.py:242-259)
and, independently of the reference, the Gaussian likelihood is checked
against ``scipy.stats.norm``.  Likelihood values / conv outputs / bpp beyond
those KATs are restatement-defined ("parity pinned by KATs, values
restatement-defined").

Noise injection
---------------
Training-mode quantisation draws U(-1/2, 1/2) noise
(entropy_models.py:163-167).  Parity tests inject identical noise tensors in
the oracle and in the HIP path through ``NoiseFeed`` (a queue of tensors in
the *logical* NCHW shape of the quantised input).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# --------------------------------------------------------------------------
# noise source
# --------------------------------------------------------------------------


class NoiseFeed:
    """Queue of noise tensors consumed, in call order, by 'noise' quantisation."""

    active: Optional["NoiseFeed"] = None

    def __init__(self, tensors: Sequence[torch.Tensor] = (), record: Optional[torch.Generator] = None):
        # record: when the queue is empty, draw from this generator and keep the
        # draws in .drawn so the identical sequence can be replayed elsewhere
        self._q = list(tensors)
        self.record = record
        self.drawn: List[torch.Tensor] = []

    def __enter__(self):
        NoiseFeed.active = self
        return self

    def __exit__(self, *exc):
        NoiseFeed.active = None

    def pop(self, shape) -> torch.Tensor:
        if not self._q and self.record is not None:
            t = torch.empty(tuple(shape)).uniform_(-0.5, 0.5, generator=self.record)
            self.drawn.append(t)
            return t
        t = self._q.pop(0)
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"injected noise shape {tuple(t.shape)} != {tuple(shape)}")
        return t


def _noise_like(x: torch.Tensor) -> torch.Tensor:
    # entropy_models.py:163-167 draws uniform_(-0.5, 0.5) of x's shape
    if NoiseFeed.active is not None:
        return NoiseFeed.active.pop(x.shape).to(device=x.device, dtype=x.dtype)
    return torch.empty_like(x).uniform_(-0.5, 0.5)


# --------------------------------------------------------------------------
# L1 ops  (ops/bound_ops.py:36-80, ops/parametrizers.py:38-64)
# --------------------------------------------------------------------------


class _LowerBoundFn(torch.autograd.Function):
    """max(x, bound); gradient passes iff x >= bound or grad < 0 (bound_ops.py:36-43)."""

    @staticmethod
    def forward(ctx, x, bound):
        ctx.save_for_backward(x, bound)
        return torch.max(x, bound)

    @staticmethod
    def backward(ctx, g):
        x, bound = ctx.saved_tensors
        keep = (x >= bound) | (g < 0)
        return keep * g, None


class LowerBound(nn.Module):
    def __init__(self, bound: float):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return _LowerBoundFn.apply(x, self.bound)


class NonNegativeParametrizer(nn.Module):
    """out = LowerBound(x)^2 - pedestal, bound = sqrt(minimum + pedestal) (parametrizers.py:38-64)."""

    def __init__(self, minimum: float = 0.0, reparam_offset: float = 2 ** -18):
        super().__init__()
        self.minimum = float(minimum)
        self.reparam_offset = float(reparam_offset)
        self.register_buffer("pedestal", torch.Tensor([self.reparam_offset ** 2]))
        self.lower_bound = LowerBound((self.minimum + self.reparam_offset ** 2) ** 0.5)

    def init(self, x):
        return torch.sqrt(torch.max(x + self.pedestal, self.pedestal))

    def forward(self, x):
        return self.lower_bound(x) ** 2 - self.pedestal


def ste_round(x):
    """ops/ops.py:35-49."""
    return torch.round(x) - x.detach() + x


# --------------------------------------------------------------------------
# L2 layers  (layers/gdn.py:41-121, layers/layers.py:52-78, models/utils.py:128-146)
# --------------------------------------------------------------------------


class GDN(nn.Module):
    """norm_i = beta_i + sum_j gamma[i,j] x_j^2 ; out = x * rsqrt(norm) (IGDN: sqrt) (gdn.py:41-92)."""

    def __init__(self, in_channels, inverse=False, beta_min=1e-6, gamma_init=0.1):
        super().__init__()
        self.inverse = bool(inverse)
        self.beta_reparam = NonNegativeParametrizer(minimum=float(beta_min))
        self.beta = nn.Parameter(self.beta_reparam.init(torch.ones(in_channels)))
        self.gamma_reparam = NonNegativeParametrizer()
        self.gamma = nn.Parameter(self.gamma_reparam.init(float(gamma_init) * torch.eye(in_channels)))

    def forward(self, x):
        C = x.shape[1]
        beta = self.beta_reparam(self.beta)
        gamma = self.gamma_reparam(self.gamma).reshape(C, C, 1, 1)
        norm = F.conv2d(x ** 2, gamma, beta)
        norm = torch.sqrt(norm) if self.inverse else torch.rsqrt(norm)
        return x * norm


class GDN1(GDN):
    """gdn.py:95-121."""

    def forward(self, x):
        C = x.shape[1]
        beta = self.beta_reparam(self.beta)
        gamma = self.gamma_reparam(self.gamma).reshape(C, C, 1, 1)
        norm = F.conv2d(torch.abs(x), gamma, beta)
        if not self.inverse:
            norm = 1.0 / norm
        return x * norm


class MaskedConv2d(nn.Conv2d):
    """layers.py:52-78 (weight masked in place every call)."""

    def __init__(self, *args, mask_type="A", **kwargs):
        super().__init__(*args, **kwargs)
        if mask_type not in ("A", "B"):
            raise ValueError(f'Invalid "mask_type" value "{mask_type}"')
        self.register_buffer("mask", torch.ones_like(self.weight.data))
        _, _, h, w = self.mask.size()
        self.mask[:, :, h // 2, w // 2 + (mask_type == "B"):] = 0
        self.mask[:, :, h // 2 + 1:] = 0

    def forward(self, x):
        self.weight.data *= self.mask
        return super().forward(x)


def conv(cin, cout, kernel_size=5, stride=2):
    """models/utils.py:128-135."""
    return nn.Conv2d(cin, cout, kernel_size=kernel_size, stride=stride, padding=kernel_size // 2)


def deconv(cin, cout, kernel_size=5, stride=2):
    """models/utils.py:138-146."""
    return nn.ConvTranspose2d(cin, cout, kernel_size=kernel_size, stride=stride,
                              output_padding=stride - 1, padding=kernel_size // 2)


# --------------------------------------------------------------------------
# L3 entropy models  (entropy_models/entropy_models.py)
# --------------------------------------------------------------------------


class EntropyModel(nn.Module):
    """entropy_models.py:101-199 (coder plumbing omitted: not on the hot path)."""

    def __init__(self, likelihood_bound=1e-9, entropy_coder=None, entropy_coder_precision=16):
        super().__init__()
        self.entropy_coder_precision = int(entropy_coder_precision)
        self.use_likelihood_bound = likelihood_bound > 0
        if self.use_likelihood_bound:
            self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())

    def forward(self, *args):
        raise NotImplementedError()

    def quantize(self, inputs, mode, means=None):
        """entropy_models.py:157-182; torch.round is half-to-even."""
        if mode not in ("noise", "dequantize", "symbols"):
            raise ValueError(f'Invalid quantization mode: "{mode}"')
        if mode == "noise":
            return inputs + _noise_like(inputs)
        out = inputs.clone()
        if means is not None:
            out -= means
        out = torch.round(out)
        if mode == "dequantize":
            if means is not None:
                out += means
            return out
        return out.int()

    @staticmethod
    def dequantize(inputs, means=None, dtype=torch.float):
        """entropy_models.py:190-199."""
        if means is not None:
            out = inputs.type_as(means)
            out += means
            return out
        return inputs.type(dtype)


class EntropyBottleneck(EntropyModel):
    """Factorized density with a per-channel monotone MLP (entropy_models.py:330-540)."""

    def __init__(self, channels, *args, tail_mass=1e-9, init_scale=10, filters=(3, 3, 3, 3), **kwargs):
        super().__init__(*args, **kwargs)
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        widths = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        for i in range(len(self.filters) + 1):
            fill = np.log(np.expm1(1 / scale / widths[i + 1]))
            m = torch.Tensor(self.channels, widths[i + 1], widths[i]).fill_(fill)
            self.register_parameter(f"_matrix{i:d}", nn.Parameter(m))
            b = torch.Tensor(self.channels, widths[i + 1], 1)
            nn.init.uniform_(b, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(b))
            if i < len(self.filters):
                f = torch.zeros(self.channels, widths[i + 1], 1)
                self.register_parameter(f"_factor{i:d}", nn.Parameter(f))
        q = torch.Tensor([-self.init_scale, 0, self.init_scale]).repeat(self.channels, 1, 1)
        self.quantiles = nn.Parameter(q)
        t = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-t, 0, t]))

    def _get_medians(self):
        return self.quantiles[:, :, 1:2]

    def _logits_cumulative(self, inputs, stop_gradient):
        """entropy_models.py:457-477."""
        h = inputs
        for i in range(len(self.filters) + 1):
            m = getattr(self, f"_matrix{i:d}")
            b = getattr(self, f"_bias{i:d}")
            if stop_gradient:
                m, b = m.detach(), b.detach()
            h = torch.matmul(F.softplus(m), h)
            h = h + b
            if i < len(self.filters):
                f = getattr(self, f"_factor{i:d}")
                if stop_gradient:
                    f = f.detach()
                h = h + torch.tanh(f) * torch.tanh(h)
        return h

    def _likelihood(self, inputs):
        """entropy_models.py:480-492 (sign is detached)."""
        lower = self._logits_cumulative(inputs - 0.5, stop_gradient=False)
        upper = self._logits_cumulative(inputs + 0.5, stop_gradient=False)
        sign = -torch.sign(lower + upper).detach()
        return torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))

    def loss(self):
        """entropy_models.py:450-454."""
        logits = self._logits_cumulative(self.quantiles, stop_gradient=True)
        return torch.abs(logits - self.target).sum()

    def forward(self, x, training=None):
        """entropy_models.py:495-540: channels first, flatten, quantise, likelihood, restore."""
        if training is None:
            training = self.training
        nd = x.dim()
        perm = list(range(nd))
        perm[0], perm[1] = perm[1], perm[0]
        inv = list(np.argsort(perm))
        xc = x.permute(*perm).contiguous()
        shape = xc.size()
        values = xc.reshape(xc.size(0), 1, -1)
        if training:
            # noise is injected in the logical (input) layout so both paths see the same values
            if NoiseFeed.active is not None:
                n = NoiseFeed.active.pop(x.shape).to(device=x.device, dtype=x.dtype)
                n = n.permute(*perm).contiguous().reshape(values.shape)
                outputs = values + n
            else:
                outputs = self.quantize(values, "noise")
        else:
            outputs = self.quantize(values, "dequantize", self._get_medians())
        lik = self._likelihood(outputs)
        if self.use_likelihood_bound:
            lik = self.likelihood_lower_bound(lik)
        outputs = outputs.reshape(shape).permute(*inv).contiguous()
        lik = lik.reshape(shape).permute(*inv).contiguous()
        return outputs, lik


class GaussianConditional(EntropyModel):
    """entropy_models.py:577-740."""

    def __init__(self, scale_table, *args, scale_bound=0.11, tail_mass=1e-9, **kwargs):
        super().__init__(*args, **kwargs)
        if not isinstance(scale_table, (type(None), list, tuple)):
            raise ValueError(f'Invalid type for scale_table "{type(scale_table)}"')
        if isinstance(scale_table, (list, tuple)) and len(scale_table) < 1:
            raise ValueError(f'Invalid scale_table length "{len(scale_table)}"')
        if scale_table and (list(scale_table) != sorted(scale_table) or any(s <= 0 for s in scale_table)):
            raise ValueError(f'Invalid scale_table "({scale_table})"')
        self.tail_mass = float(tail_mass)
        if scale_bound is None and scale_table:
            scale_bound = scale_table[0]
        if scale_bound is None or scale_bound <= 0:
            raise ValueError("Invalid parameters")
        self.lower_bound_scale = LowerBound(scale_bound)
        self.register_buffer("scale_table",
                             torch.Tensor(tuple(float(s) for s in scale_table)) if scale_table else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]))

    @staticmethod
    def _standardized_cumulative(x):
        """entropy_models.py:629-635: Phi(x) = 0.5 erfc(-x/sqrt(2))."""
        return 0.5 * torch.erfc(float(-(2 ** -0.5)) * x)

    def _likelihood(self, inputs, scales, means=None):
        """entropy_models.py:692-709."""
        values = inputs - means if means is not None else inputs
        scales = self.lower_bound_scale(scales)
        values = torch.abs(values)
        upper = self._standardized_cumulative((0.5 - values) / scales)
        lower = self._standardized_cumulative((-0.5 - values) / scales)
        return upper - lower

    def forward(self, inputs, scales, means=None, training=None):
        """entropy_models.py:715-731."""
        if training is None:
            training = self.training
        outputs = self.quantize(inputs, "noise" if training else "dequantize", means)
        lik = self._likelihood(outputs, scales, means)
        if self.use_likelihood_bound:
            lik = self.likelihood_lower_bound(lik)
        return outputs, lik

    def build_indexes(self, scales):
        """entropy_models.py:735-740."""
        scales = self.lower_bound_scale(scales)
        idx = scales.new_full(scales.size(), len(self.scale_table) - 1).int()
        for s in self.scale_table[:-1]:
            idx -= (scales <= s).int()
        return idx


# --------------------------------------------------------------------------
# L4 models  (models/google.py)
# --------------------------------------------------------------------------

SCALES_MIN, SCALES_MAX, SCALES_LEVELS = 0.11, 256, 64


def get_scale_table(min=SCALES_MIN, max=SCALES_MAX, levels=SCALES_LEVELS):
    """google.py:208-214."""
    return torch.exp(torch.linspace(math.log(min), math.log(max), levels))


class CompressionModel(nn.Module):
    """google.py:58-123."""

    def __init__(self, entropy_bottleneck_channels, init_weights=None):
        super().__init__()
        self.entropy_bottleneck = EntropyBottleneck(entropy_bottleneck_channels)

    def aux_loss(self):
        return sum(m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck))

    def forward(self, *args):
        raise NotImplementedError()


def _analysis(channel, N, M):
    return nn.Sequential(conv(channel, N), GDN(N), conv(N, N), GDN(N), conv(N, N), GDN(N), conv(N, M))


def _synthesis(channel, N, M):
    return nn.Sequential(deconv(M, N), GDN(N, inverse=True), deconv(N, N), GDN(N, inverse=True),
                         deconv(N, N), GDN(N, inverse=True), deconv(N, channel))


class FactorizedPrior(CompressionModel):
    """google.py:127-204 (forward :172-182)."""

    def __init__(self, N, M, channel=3, **kwargs):
        super().__init__(entropy_bottleneck_channels=M, **kwargs)
        self.g_a = _analysis(channel, N, M)
        self.g_s = _synthesis(channel, N, M)
        self.N, self.M = N, M

    def forward(self, x):
        y = self.g_a(x)
        y_hat, y_lik = self.entropy_bottleneck(y)
        return {"x_hat": self.g_s(y_hat), "likelihoods": {"y": y_lik}}


class ScaleHyperprior(CompressionModel):
    """google.py:218-344 (forward :281-295)."""

    def __init__(self, N, M, channel=3, **kwargs):
        super().__init__(entropy_bottleneck_channels=N, **kwargs)
        self.g_a = _analysis(channel, N, M)
        self.g_s = _synthesis(channel, N, M)
        self.h_a = nn.Sequential(conv(M, N, stride=1, kernel_size=3), nn.ReLU(inplace=True),
                                 conv(N, N), nn.ReLU(inplace=True), conv(N, N))
        self.h_s = nn.Sequential(deconv(N, N), nn.ReLU(inplace=True), deconv(N, N), nn.ReLU(inplace=True),
                                 conv(N, M, stride=1, kernel_size=3), nn.ReLU(inplace=True))
        self.gaussian_conditional = GaussianConditional(None)
        self.N, self.M = int(N), int(M)

    def forward(self, x):
        y = self.g_a(x)
        z = self.h_a(torch.abs(y))
        z_hat, z_lik = self.entropy_bottleneck(z)
        scales_hat = self.h_s(z_hat)
        y_hat, y_lik = self.gaussian_conditional(y, scales_hat)
        return {"x_hat": self.g_s(y_hat), "likelihoods": {"y": y_lik, "z": z_lik}}


class MeanScaleHyperprior(ScaleHyperprior):
    """google.py:348-416 (forward :379-391)."""

    def __init__(self, N, M, channel=3, **kwargs):
        super().__init__(N, M, channel, **kwargs)
        self.h_a = nn.Sequential(conv(M, N, stride=1, kernel_size=3), nn.LeakyReLU(inplace=True),
                                 conv(N, N), nn.LeakyReLU(inplace=True), conv(N, N))
        self.h_s = nn.Sequential(deconv(N, M), nn.LeakyReLU(inplace=True), deconv(M, M * 3 // 2),
                                 nn.LeakyReLU(inplace=True), conv(M * 3 // 2, M * 2, stride=1, kernel_size=3))

    def forward(self, x):
        y = self.g_a(x)
        z = self.h_a(y)
        z_hat, z_lik = self.entropy_bottleneck(z)
        scales_hat, means_hat = self.h_s(z_hat).chunk(2, 1)
        y_hat, y_lik = self.gaussian_conditional(y, scales_hat, means=means_hat)
        return {"x_hat": self.g_s(y_hat), "likelihoods": {"y": y_lik, "z": z_lik}}


class JointAutoregressiveHierarchicalPriors(MeanScaleHyperprior):
    """google.py:421-515 (forward :493-515)."""

    def __init__(self, N=192, M=192, channel=3, **kwargs):
        super().__init__(N=N, M=M, channel=channel, **kwargs)
        self.entropy_parameters = nn.Sequential(
            nn.Conv2d(M * 12 // 3, M * 10 // 3, 1), nn.LeakyReLU(inplace=True),
            nn.Conv2d(M * 10 // 3, M * 8 // 3, 1), nn.LeakyReLU(inplace=True),
            nn.Conv2d(M * 8 // 3, M * 6 // 3, 1))
        self.context_prediction = MaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)

    def forward(self, x):
        y = self.g_a(x)
        z = self.h_a(y)
        z_hat, z_lik = self.entropy_bottleneck(z)
        params = self.h_s(z_hat)
        y_hat = self.gaussian_conditional.quantize(y, "noise" if self.training else "dequantize")
        ctx = self.context_prediction(y_hat)
        scales_hat, means_hat = self.entropy_parameters(torch.cat((params, ctx), dim=1)).chunk(2, 1)
        _, y_lik = self.gaussian_conditional(y, scales_hat, means=means_hat)
        return {"x_hat": self.g_s(y_hat), "likelihoods": {"y": y_lik, "z": z_lik}}


# --------------------------------------------------------------------------
# cheng2020 building blocks (layers/layers.py:81-244) and models
# (models/waseda.py:48-158)
# --------------------------------------------------------------------------


def conv3x3(cin, cout, stride=1):
    """layers.py:81-83."""
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1)


def conv1x1(cin, cout, stride=1):
    """layers.py:94-96."""
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride)


def subpel_conv3x3(cin, cout, r=1):
    """layers.py:86-91: conv to cout*r^2 channels + PixelShuffle(r)."""
    return nn.Sequential(nn.Conv2d(cin, cout * r * r, kernel_size=3, padding=1), nn.PixelShuffle(r))


class ResidualBlockWithStride(nn.Module):
    """layers.py:97-129."""

    def __init__(self, cin, cout, stride=2):
        super().__init__()
        self.conv1 = conv3x3(cin, cout, stride=stride)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(cout, cout)
        self.gdn = GDN(cout)
        self.skip = conv1x1(cin, cout, stride=stride) if (stride != 1 or cin != cout) else None

    def forward(self, x):
        out = self.gdn(self.conv2(self.leaky_relu(self.conv1(x))))
        identity = self.skip(x) if self.skip is not None else x
        return out + identity


class ResidualBlockUpsample(nn.Module):
    """layers.py:132-159."""

    def __init__(self, cin, cout, upsample=2):
        super().__init__()
        self.subpel_conv = subpel_conv3x3(cin, cout, upsample)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv = conv3x3(cout, cout)
        self.igdn = GDN(cout, inverse=True)
        self.upsample = subpel_conv3x3(cin, cout, upsample)

    def forward(self, x):
        out = self.igdn(self.conv(self.leaky_relu(self.subpel_conv(x))))
        return out + self.upsample(x)


class ResidualBlock(nn.Module):
    """layers.py:162-193."""

    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = conv3x3(cin, cout)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(cout, cout)
        self.skip = conv1x1(cin, cout) if cin != cout else None

    def forward(self, x):
        out = self.leaky_relu(self.conv2(self.leaky_relu(self.conv1(x))))
        identity = self.skip(x) if self.skip is not None else x
        return out + identity


class ResidualUnit(nn.Module):
    """layers.py:211-226 (defined inside AttentionBlock.__init__ in the reference)."""

    def __init__(self, N):
        super().__init__()
        self.conv = nn.Sequential(conv1x1(N, N // 2), nn.ReLU(inplace=True), conv3x3(N // 2, N // 2),
                                  nn.ReLU(inplace=True), conv1x1(N // 2, N))
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.relu(self.conv(x) + x)


class AttentionBlock(nn.Module):
    """layers.py:196-244."""

    def __init__(self, N):
        super().__init__()
        self.conv_a = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N))
        self.conv_b = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N), conv1x1(N, N))

    def forward(self, x):
        return self.conv_a(x) * torch.sigmoid(self.conv_b(x)) + x


class Cheng2020Anchor(JointAutoregressiveHierarchicalPriors):
    """waseda.py:48-123: residual analysis/synthesis, 3x3 hyper transforms, sub-pixel upsampling."""

    def __init__(self, N=192, channel=3, **kwargs):
        super().__init__(N=N, M=N, **kwargs)
        self.g_a = nn.Sequential(
            ResidualBlockWithStride(channel, N, stride=2), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), ResidualBlock(N, N), conv3x3(N, N, stride=2))
        self.h_a = nn.Sequential(
            conv3x3(N, N), nn.LeakyReLU(inplace=True), conv3x3(N, N), nn.LeakyReLU(inplace=True),
            conv3x3(N, N, stride=2), nn.LeakyReLU(inplace=True), conv3x3(N, N), nn.LeakyReLU(inplace=True),
            conv3x3(N, N, stride=2))
        self.h_s = nn.Sequential(
            conv3x3(N, N), nn.LeakyReLU(inplace=True), subpel_conv3x3(N, N, 2), nn.LeakyReLU(inplace=True),
            conv3x3(N, N * 3 // 2), nn.LeakyReLU(inplace=True), subpel_conv3x3(N * 3 // 2, N * 3 // 2, 2),
            nn.LeakyReLU(inplace=True), conv3x3(N * 3 // 2, N * 2))
        self.g_s = nn.Sequential(
            ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N),
            ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2),
            ResidualBlock(N, N), subpel_conv3x3(N, channel, 2))


class Cheng2020Attention(Cheng2020Anchor):
    """waseda.py:126-158: Anchor + attention blocks in g_a / g_s."""

    def __init__(self, N=192, channel=3, **kwargs):
        super().__init__(N=N, **kwargs)
        self.g_a = nn.Sequential(
            ResidualBlockWithStride(channel, N, stride=2), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), AttentionBlock(N), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), ResidualBlock(N, N), conv3x3(N, N, stride=2),
            AttentionBlock(N))
        self.g_s = nn.Sequential(
            AttentionBlock(N), ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N),
            ResidualBlockUpsample(N, N, 2), AttentionBlock(N), ResidualBlock(N, N),
            ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N), subpel_conv3x3(N, channel, 2))


# --------------------------------------------------------------------------
# L7 caller: RD loss, optimizer split, one training step (examples/train.py)
# --------------------------------------------------------------------------

LMBDA = [256, 512, 1024, 2048, 4096, 8192, 10240]   # train.py:65


class RateDistortionLoss(nn.Module):
    """train.py:59-82: bpp = sum_k sum log(lik_k)/(-ln2 N H W); loss = lmbda[q] * mse + bpp."""

    def __init__(self, q):
        super().__init__()
        self.q = q

    def forward(self, output, target):
        N, _, H, W = target.size()
        npix = N * H * W
        out = {"bpp_loss": sum(torch.log(l).sum() / (-math.log(2) * npix)
                               for l in output["likelihoods"].values())}
        out["mse_loss"] = F.mse_loss(output["x_hat"], target)
        out["loss"] = LMBDA[self.q] * out["mse_loss"] + out["bpp_loss"]
        return out


def configure_optimizers(net, lr=1e-4, aux_lr=1e-3):
    """train.py:111-142: Adam on everything but `.quantiles`, Adam(aux) on `.quantiles`."""
    named = dict(net.named_parameters())
    main = sorted(n for n, p in named.items() if not n.endswith(".quantiles") and p.requires_grad)
    aux = sorted(n for n, p in named.items() if n.endswith(".quantiles") and p.requires_grad)
    return (torch.optim.Adam((named[n] for n in main), lr=lr),
            torch.optim.Adam((named[n] for n in aux), lr=aux_lr))


def train_step(net, criterion, x, optimizer, aux_optimizer, clip_max_norm=1.0):
    """train.py:155-186 step body (fp32: autocast/GradScaler are no-ops on CPU tensors)."""
    optimizer.zero_grad()
    aux_optimizer.zero_grad()
    out = net(x)
    crit = criterion(out, x)
    crit["loss"].backward()
    if clip_max_norm > 0:
        torch.nn.utils.clip_grad_norm_(net.parameters(), clip_max_norm)
    optimizer.step()
    aux = net.aux_loss()
    aux.backward()
    aux_optimizer.step()
    return crit, aux


# --------------------------------------------------------------------------
# L5 registry (zoo/image.py:52-59,189-246)
# --------------------------------------------------------------------------

CFGS = {
    "bmshj2018-factorized": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "bmshj2018-hyperprior": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "mbt2018-mean": {q: ((128, 192) if q <= 4 else (192, 320)) for q in range(1, 9)},
    "mbt2018": {q: ((192, 192) if q <= 4 else (192, 320)) for q in range(1, 9)},
    "cheng2020-anchor": {q: ((128,) if q <= 3 else (192,)) for q in range(1, 7)},
    "cheng2020-attn": {q: ((128,) if q <= 3 else (192,)) for q in range(1, 7)},
}
ARCHS = {
    "bmshj2018-factorized": FactorizedPrior,
    "bmshj2018-hyperprior": ScaleHyperprior,
    "mbt2018-mean": MeanScaleHyperprior,
    "mbt2018": JointAutoregressiveHierarchicalPriors,
    "cheng2020-anchor": Cheng2020Anchor,
    "cheng2020-attn": Cheng2020Attention,
}


def build(name: str, quality: int, channel: int = 3) -> CompressionModel:
    return ARCHS[name](*CFGS[name][quality], channel=channel)


# --------------------------------------------------------------------------
# eval helpers (utils/eval_model/__main__t.py:88-91,149-211)
# --------------------------------------------------------------------------


def psnr(a, b):
    mse = F.mse_loss(a, b).item()
    return -10 * math.log10(mse)


@torch.no_grad()
def entropy_estimation(net, x):
    """__main__t.py:149-211 inner part: eval-mode forward, bpp over the (unpadded) pixel count."""
    out = net(x)
    N, _, H, W = x.shape
    npix = N * H * W
    bpp = sum(torch.log(l).sum() / (-math.log(2) * npix) for l in out["likelihoods"].values())
    return {"bpp": float(bpp), "psnr": psnr(out["x_hat"], x), "x_hat": out["x_hat"]}   # no clamp: __main__t.py:169,207
