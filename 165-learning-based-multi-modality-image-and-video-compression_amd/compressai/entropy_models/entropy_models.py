"""EntropyModel / EntropyBottleneck / GaussianConditional on the HIP kernels.

Reference: compressai/entropy_models/entropy_models.py (quantize :157-182,
EntropyBottleneck :330-574, GaussianConditional :577-740).  Parameters,
buffers, constructor arguments, ValueError checks and the
``forward(...) -> (outputs, likelihoods)`` contract are kept; the forward
and backward of the likelihood path are single fused kernels
(cai_eb_fwd/_bwd, cai_gc_fwd/_bwd) instead of ~40 small torch ops, and
training-mode noise is U(-1/2, 1/2) as in the reference
(``empty_like(x).uniform_(-0.5, 0.5)``, entropy_models.py:170), drawn on the
device by cai_uniform_noise (Philox4x32-10, counter kept in device memory: a
captured graph draws new noise on every replay without torch's generator and
its per-replay re-seeding launches); seeded from torch.cuda.initial_seed(), so
torch.cuda.manual_seed() keeps runs reproducible.  By default no launch of its
own makes the draw: the first kernel that consumes it generates it in-register
(_ops.DeviceDraw, cai_noise_src DRAW) and the later ones regenerate it (REPLAY),
the same values cai_uniform_noise would have written (CAI_FUSED_NOISE=0: the
separate draw).  Tests inject their own draws (set_noise_source) to compare
against the CPU oracle.

The bitstream side follows the reference too:
update() evaluates the pmfs with the reference's torch expressions on the
module's device and quantizes them to CDF tables in libcai_coder.so
(cai_pmf_to_quantized_cdf_rows); compress() takes its integer symbols from
the quantize kernel (SYMBOLS mode) and codes one rANS stream per image on
host threads (cai_rans_encode_batch), byte-identical to compressai.ans;
decompress() decodes them (cai_rans_decode_batch) and dequantizes.
"""
from __future__ import annotations

import ctypes
import os
from typing import Any, Callable, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.nn as nn

import scipy.stats

from .. import _coder
from .._native import F32, NOISE_STATE_WORDS, Q_DEQUANTIZE, Q_NOISE, Q_SYMBOLS, lib
from .._ops import (BottleneckAuxFn, BottleneckFn, DeviceDraw, GaussianFn, _check_cuda, _p, _stream, as_rows, dcode,
                    empty_rows_like, noise_src)
from ..ops import LowerBound

__all__ = ["EntropyModel", "EntropyBottleneck", "GaussianConditional", "set_noise_source", "seed_noise"]

# ---------------------------------------------------------------------------
# noise source: torch's generator by default; tests inject identical tensors
# into this build and into the CPU oracle.
# ---------------------------------------------------------------------------
_noise_source: Optional[Callable[[torch.Tensor], torch.Tensor]] = None


def set_noise_source(fn: Optional[Callable[[torch.Tensor], torch.Tensor]]):
    """fn(x) -> fp32 noise tensor of x's logical shape (None restores U(-1/2,1/2))."""
    global _noise_source
    _noise_source = fn


# on-device generator state per GPU: [seed, draw index, arrival ticket, ..., the DRAW launches' per-XCD arrival
# shards] (NOISE_STATE_WORDS uint64 bit patterns, include/cai.h).  ONE state per device: draws that use it must
# be ordered (one stream, or event-ordered) -- two concurrent launches would read the same draw index and mix
# their arrival tickets.  The models' hyper-branch fork therefore draws z's noise on the caller's stream before
# forking (models/google.py, _z_noise).
_noise_states: dict = {}
# A/B knobs (read once): CAI_TORCH_NOISE=1 draws with torch's generator instead (`uniform_`, as the reference);
# CAI_FUSED_NOISE=0 draws into a buffer with cai_uniform_noise instead of inside the consuming kernel
_TORCH_NOISE = os.environ.get("CAI_TORCH_NOISE", "0") == "1"
_FUSED_NOISE = os.environ.get("CAI_FUSED_NOISE", "1") == "1"


def _as_i64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def seed_noise(seed: int, device=None) -> None:
    """Seed the training-noise generator of `device` (default: the current GPU) and restart its stream."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _noise_states.get(idx)
    if st is None:
        st = [None, None]
        _noise_states[idx] = st
    if st[0] is None:
        st[0] = torch.zeros(NOISE_STATE_WORDS, dtype=torch.int64, device=torch.device("cuda", idx))
    st[0].zero_()
    st[0][0].fill_(_as_i64(seed))
    with torch.cuda.device(idx):
        st[1] = torch.cuda.initial_seed()   # torch's seed at this point: a later manual_seed() re-seeds


def _noise_state(dev: torch.device) -> torch.Tensor:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _noise_states.get(idx)
    seed = None
    if not torch.cuda.is_current_stream_capturing():
        with torch.cuda.device(idx):
            seed = torch.cuda.initial_seed()
    # (re)seed on first use and whenever torch.cuda.manual_seed() changed the device seed (eager mode; a
    # capture keeps the state it finds)
    if st is None and seed is None:
        raise RuntimeError("training noise: run one eager training-mode forward (or call seed_noise()) before "
                           "capturing a graph; the generator state must exist outside the capture")
    if st is None or (seed is not None and seed != st[1]):
        seed_noise(seed, torch.device("cuda", idx))
        st = _noise_states[idx]
    return st[0]


def _draw_noise(x: torch.Tensor) -> torch.Tensor:
    if _noise_source is not None:
        n = _noise_source(x)
        if tuple(n.shape) != tuple(x.shape):
            raise ValueError(f"noise source returned shape {tuple(n.shape)}, expected {tuple(x.shape)}")
        return n.to(device=x.device, dtype=torch.float32)
    if _TORCH_NOISE:
        return torch.empty_like(x, dtype=torch.float32).uniform_(-0.5, 0.5)
    _check_cuda(x)
    out = torch.empty_like(x, dtype=torch.float32)   # dense storage: numel() values from data_ptr()
    lib.cai_uniform_noise(_p(out), out.numel(), _p(_noise_state(x.device)), _stream())
    return out


def _noise_for(x: torch.Tensor):
    """Training noise for x, to hand to a noise-mode entropy kernel: a DeviceDraw (drawn inside that kernel),
    or -- with an injected source, torch's generator, or CAI_FUSED_NOISE=0 -- a tensor from _draw_noise."""
    if _noise_source is not None or _TORCH_NOISE or not _FUSED_NOISE:
        return _draw_noise(x)
    _check_cuda(x)
    return DeviceDraw(x.shape, _noise_state(x.device))


class _QuantizeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, means, noise, mode: int):
        """noise: None, an fp32 tensor, or a DeviceDraw (NOISE mode)."""
        draw = isinstance(noise, DeviceDraw)
        _check_cuda(x, means, None if draw else noise)
        xr, xld, npix, C = as_rows(x)
        m = None
        mld, mpc = 0, 0
        if means is not None:
            if means.numel() == C and means.dim() != x.dim():
                m, mld, mpc = means.float().contiguous().reshape(C), 0, 1
            else:
                m, mld = as_rows(means.float().expand_as(x))[:2]
        nr, nld = (None, 0) if noise is None or draw else as_rows(noise)[:2]
        odt = torch.int32 if mode == Q_SYMBOLS else x.dtype
        out, obuf = empty_rows_like(x.shape, odt, x.device)
        lib.cai_quantize(mode, npix, C, _p(xr), dcode(x.dtype), xld, _p(m), mld, mpc, noise_src(noise, nr, nld),
                         _p(obuf), dcode(x.dtype) if mode != Q_SYMBOLS else F32, C, _stream())
        ctx.mode = mode
        ctx.has_means = means is not None
        ctx.mshape = None if means is None else means.shape
        return out

    @staticmethod
    def backward(ctx, g):
        if ctx.mode == Q_NOISE:
            return g, None, None, None
        gm = None
        if ctx.has_means:
            gm = g.float()
            if tuple(gm.shape) != tuple(ctx.mshape):
                gm = gm.sum_to_size(ctx.mshape)
        return torch.zeros_like(g), gm, None, None


class EntropyModel(nn.Module):
    def __init__(self, likelihood_bound: float = 1e-9, entropy_coder: Optional[str] = None,
                 entropy_coder_precision: int = 16):
        super().__init__()
        from .. import available_entropy_coders, get_entropy_coder

        if entropy_coder is None:
            entropy_coder = get_entropy_coder()
        if not isinstance(entropy_coder, str):
            raise ValueError(f'Invalid method type "{type(entropy_coder)}"')
        if entropy_coder not in available_entropy_coders():
            raise ValueError(f'Unknown entropy coder "{entropy_coder}" (available: {", ".join(available_entropy_coders())})')
        self.entropy_coder = entropy_coder
        self.entropy_coder_precision = int(entropy_coder_precision)
        self.use_likelihood_bound = likelihood_bound > 0
        # python-side copy: kernels take the bound by value (no .item() sync, graph-capturable)
        self._lik_bound_value = float(likelihood_bound) if self.use_likelihood_bound else 0.0
        if self.use_likelihood_bound:
            self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())

    @property
    def offset(self):
        return self._offset

    @property
    def quantized_cdf(self):
        return self._quantized_cdf

    @property
    def cdf_length(self):
        return self._cdf_length

    def _lik_bound(self) -> float:
        return self._lik_bound_value

    def forward(self, *args: Any) -> Any:
        raise NotImplementedError()

    def quantize(self, inputs: torch.Tensor, mode: str, means: Optional[torch.Tensor] = None) -> torch.Tensor:
        if mode not in ("noise", "dequantize", "symbols"):
            raise ValueError(f'Invalid quantization mode: "{mode}"')
        if mode == "noise":
            return _QuantizeFn.apply(inputs, None, _noise_for(inputs), Q_NOISE)
        if mode == "dequantize":
            return _QuantizeFn.apply(inputs, means, None, Q_DEQUANTIZE)
        return _QuantizeFn.apply(inputs, means, None, Q_SYMBOLS)

    @staticmethod
    def dequantize(inputs: torch.Tensor, means: Optional[torch.Tensor] = None, dtype: torch.dtype = torch.float):
        if means is not None:
            out = inputs.type_as(means)
            out += means
            return out
        return inputs.type(dtype)

    # ---- bitstream side (entropy_models.py:206-327) --------------------------

    def _pmf_to_cdf(self, pmf, tail_mass, pmf_length, max_length):
        """entropy_models.py:206-214: row i = quantized CDF of [pmf[i, :pmf_length[i]], tail_mass[i]]
        in a zero-filled [rows, max_length + 2] int32 table (libcai_coder.so, rows on host threads)."""
        lengths = pmf_length.detach().reshape(-1).to("cpu", torch.int64).numpy()
        rows = lengths.size
        p = pmf.detach().float().reshape(rows, -1).cpu().numpy()
        tail = tail_mass.detach().float().reshape(rows, -1)[:, 0].cpu().numpy()
        table = np.zeros((rows, max_length + 1), dtype=np.float32)
        keep = np.arange(p.shape[1])[None, :] < lengths[:, None]
        table[:, :p.shape[1]] = np.where(keep, p, 0.0)
        table[np.arange(rows), lengths] = tail
        cdf = _coder.pmf_to_quantized_cdf_rows(table, lengths + 1, self.entropy_coder_precision, max_length + 2)
        return torch.from_numpy(cdf).to(pmf.device)

    def _check_cdf_size(self):
        if self._quantized_cdf.numel() == 0:
            raise ValueError("Uninitialized CDFs. Run update() first")
        if len(self._quantized_cdf.size()) != 2:
            raise ValueError(f"Invalid CDF size {self._quantized_cdf.size()}")

    def _check_offsets_size(self):
        if self._offset.numel() == 0:
            raise ValueError("Uninitialized offsets. Run update() first")
        if len(self._offset.size()) != 1:
            raise ValueError(f"Invalid offsets size {self._offset.size()}")

    def _check_cdf_length(self):
        if self._cdf_length.numel() == 0:
            raise ValueError("Uninitialized CDF lengths. Run update() first")
        if len(self._cdf_length.size()) != 1:
            raise ValueError(f"Invalid offsets size {self._cdf_length.size()}")

    def _tables(self) -> "_coder.Tables":
        return _coder.Tables(self._quantized_cdf.cpu().numpy(), self._cdf_length.reshape(-1).cpu().numpy(),
                             self._offset.reshape(-1).cpu().numpy())

    def compress(self, inputs, indexes, means=None):
        """entropy_models.py:237-270: one rANS string per batch element."""
        if len(inputs.size()) < 2:
            raise ValueError("Invalid `inputs` size. Expected a tensor with at least 2 dimensions.")
        if inputs.size() != indexes.size():
            raise ValueError("`inputs` and `indexes` should have the same size.")
        self._check_cdf_size()
        self._check_cdf_length()
        self._check_offsets_size()
        symbols = self.quantize(inputs, "symbols", means)
        B = symbols.size(0)
        sym = symbols.reshape(B, -1).cpu().numpy()
        idx = indexes.reshape(B, -1).int().cpu().numpy()
        return _coder.encode_streams(sym, idx, self._tables(), B)

    def decompress(self, strings, indexes, dtype: torch.dtype = torch.float, means: torch.Tensor = None):
        """entropy_models.py:272-327."""
        if not isinstance(strings, (tuple, list)):
            raise ValueError("Invalid `strings` parameter type.")
        if not len(strings) == indexes.size(0):
            raise ValueError("Invalid strings or indexes parameters")
        if len(indexes.size()) < 2:
            raise ValueError("Invalid `indexes` size. Expected a tensor with at least 2 dimensions.")
        self._check_cdf_size()
        self._check_cdf_length()
        self._check_offsets_size()
        if means is not None:
            if means.size()[:2] != indexes.size()[:2]:
                raise ValueError("Invalid means or indexes parameters")
            if means.size() != indexes.size():
                for i in range(2, len(indexes.size())):
                    if means.size(i) != 1:
                        raise ValueError("Invalid means parameters")
        vals = _coder.decode_streams(strings, indexes.reshape(len(strings), -1).int().cpu().numpy(), self._tables())
        outputs = torch.from_numpy(vals).to(self._quantized_cdf.device).reshape(indexes.size())
        return self.dequantize(outputs, means, dtype)


class EntropyBottleneck(EntropyModel):
    _offset: torch.Tensor

    def __init__(self, channels: int, *args: Any, tail_mass: float = 1e-9, init_scale: float = 10,
                 filters: Tuple[int, ...] = (3, 3, 3, 3), **kwargs: Any):
        super().__init__(*args, **kwargs)
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        if self.filters != (3, 3, 3, 3):
            raise ValueError("the fused EntropyBottleneck kernel implements filters=(3, 3, 3, 3)")
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        widths = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        for i in range(len(self.filters) + 1):
            init = np.log(np.expm1(1 / scale / widths[i + 1]))
            self.register_parameter(f"_matrix{i:d}",
                                    nn.Parameter(torch.Tensor(self.channels, widths[i + 1], widths[i]).fill_(init)))
            b = torch.Tensor(self.channels, widths[i + 1], 1)
            nn.init.uniform_(b, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(b))
            if i < len(self.filters):
                self.register_parameter(f"_factor{i:d}", nn.Parameter(torch.zeros(self.channels, widths[i + 1], 1)))
        self.quantiles = nn.Parameter(
            torch.Tensor([-self.init_scale, 0, self.init_scale]).repeat(self.channels, 1, 1))
        target = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _params(self) -> List[torch.Tensor]:
        return ([getattr(self, f"_matrix{i}") for i in range(5)] + [getattr(self, f"_bias{i}") for i in range(5)]
                + [getattr(self, f"_factor{i}") for i in range(4)])

    def _get_medians(self) -> torch.Tensor:
        return self.quantiles[:, :, 1:2]

    def loss(self) -> torch.Tensor:
        return BottleneckAuxFn.apply(self.quantiles, self.target, *self._params())

    def forward(self, x: torch.Tensor, training: Optional[bool] = None, noise: Optional[torch.Tensor] = None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        """noise: the U(-1/2, 1/2) draw to use in training mode (the models' concurrent forward draws it on the
        caller's stream before forking the hyper branch, so every draw of a step runs on one stream); None
        draws it here, as the reference does (entropy_models.py:495-540)."""
        if training is None:
            training = self.training
        if x.dim() < 2 or x.shape[1] != self.channels:
            raise ValueError(f"expected [B, {self.channels}, ...] input, got {tuple(x.shape)}")
        if training and noise is None:
            noise = _noise_for(x)
        elif training and tuple(noise.shape) != tuple(x.shape):
            raise ValueError(f"noise shape {tuple(noise.shape)} does not match the input's {tuple(x.shape)}")
        elif not training:
            noise = None
        return BottleneckFn.apply(x, self.quantiles, noise, Q_NOISE if training else Q_DEQUANTIZE,
                                  self._lik_bound(), *self._params())

    @staticmethod
    def _build_indexes(size):
        dims = len(size)
        view_dims = np.ones((dims,), dtype=np.int64)
        view_dims[1] = -1
        return torch.arange(size[1]).view(*view_dims).int().repeat(size[0], 1, *size[2:])

    @staticmethod
    def _extend_ndims(tensor, n):
        return tensor.reshape(-1, *([1] * n)) if n > 0 else tensor.reshape(-1)

    def _logits_cumulative(self, inputs: torch.Tensor, stop_gradient: bool) -> torch.Tensor:
        """entropy_models.py:457-477 in torch ops, for update() only (the training / eval
        forward runs the fused cai_eb_* kernels)."""
        logits = inputs
        for i in range(len(self.filters) + 1):
            matrix = getattr(self, f"_matrix{i:d}")
            bias = getattr(self, f"_bias{i:d}")
            if stop_gradient:
                matrix, bias = matrix.detach(), bias.detach()
            logits = torch.matmul(torch.nn.functional.softplus(matrix), logits) + bias
            if i < len(self.filters):
                factor = getattr(self, f"_factor{i:d}")
                if stop_gradient:
                    factor = factor.detach()
                logits = logits + torch.tanh(factor) * torch.tanh(logits)
        return logits

    @torch.no_grad()
    def update(self, force: bool = False) -> bool:
        """entropy_models.py:396-441."""
        if self._offset.numel() > 0 and not force:
            return False
        medians = self.quantiles[:, 0, 1]
        minima = torch.clamp(torch.ceil(medians - self.quantiles[:, 0, 0]).int(), min=0)
        maxima = torch.clamp(torch.ceil(self.quantiles[:, 0, 2] - medians).int(), min=0)
        self._offset = -minima
        pmf_start = medians - minima
        pmf_length = maxima + minima + 1
        max_length = int(pmf_length.max().item())
        samples = torch.arange(max_length, device=pmf_start.device)
        samples = samples[None, :] + pmf_start[:, None, None]
        half = float(0.5)
        lower = self._logits_cumulative(samples - half, stop_gradient=True)
        upper = self._logits_cumulative(samples + half, stop_gradient=True)
        sign = -torch.sign(lower + upper)
        pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
        tail_mass = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
        self._quantized_cdf = self._pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
        self._cdf_length = pmf_length + 2
        return True

    def compress(self, x):
        """entropy_models.py:559-567."""
        indexes = self._build_indexes(x.size()).to(x.device)
        medians = self._get_medians().detach()
        spatial_dims = len(x.size()) - 2
        medians = self._extend_ndims(medians, spatial_dims)
        medians = medians.expand(x.size(0), *([-1] * (spatial_dims + 1)))
        return super().compress(x, indexes, medians)

    def decompress(self, strings, size):
        """entropy_models.py:569-574."""
        output_size = (len(strings), self._quantized_cdf.size(0), *size)
        indexes = self._build_indexes(output_size).to(self._quantized_cdf.device)
        medians = self._extend_ndims(self._get_medians().detach(), len(size))
        medians = medians.expand(len(strings), *([-1] * (len(size) + 1)))
        return super().decompress(strings, indexes, medians.dtype, medians)


class GaussianConditional(EntropyModel):
    def __init__(self, scale_table: Optional[Union[List, Tuple]], *args: Any, scale_bound: float = 0.11,
                 tail_mass: float = 1e-9, **kwargs: Any):
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
        self._scale_bound_value = float(scale_bound)
        self.register_buffer("scale_table",
                             torch.Tensor(tuple(float(s) for s in scale_table)) if scale_table else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]))

    @staticmethod
    def _prepare_scale_table(scale_table):
        return torch.Tensor(tuple(float(s) for s in scale_table))

    def forward(self, inputs: torch.Tensor, scales: torch.Tensor, means: Optional[torch.Tensor] = None,
                training: Optional[bool] = None, noise: Optional[torch.Tensor] = None, scales_relu: bool = False
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        """noise: the U(-1/2, 1/2) draw to use in training mode (the models' concurrent forward shares one
        draw between g_s's input and this likelihood); None draws it here, as the reference does.
        scales_relu: the scales are the output of a ReLU whose backward mask this op applies (the producer ran
        with act_bwd_downstream: ScaleHyperprior's h_s)."""
        if training is None:
            training = self.training
        # the reference's _likelihood broadcasts scales / means against the inputs (entropy_models.py:692-709)
        try:
            if scales.shape != inputs.shape:
                scales = scales.expand_as(inputs)
            if means is not None and means.shape != inputs.shape:
                means = means.expand_as(inputs)
        except RuntimeError as e:
            raise ValueError(f"scales / means do not broadcast to the inputs' shape {tuple(inputs.shape)}") from e
        if training and noise is None:
            noise = _noise_for(inputs)
        elif not training:
            noise = None
        sb = self._scale_bound_value
        return GaussianFn.apply(inputs, scales, means, noise, Q_NOISE if training else Q_DEQUANTIZE, sb,
                                self._lik_bound(), bool(scales_relu))

    def build_indexes(self, scales: torch.Tensor) -> torch.Tensor:
        scales = torch.clamp_min(scales, self._scale_bound_value)
        indexes = scales.new_full(scales.size(), len(self.scale_table) - 1).int()
        for s in self.scale_table[:-1]:
            indexes -= (scales <= s).int()
        return indexes

    @staticmethod
    def _standardized_cumulative(inputs: torch.Tensor) -> torch.Tensor:
        """entropy_models.py:629-635 (update() only; the likelihood kernels use the same erfc form)."""
        half = float(0.5)
        const = float(-(2 ** -0.5))
        return half * torch.erfc(const * inputs)

    @staticmethod
    def _standardized_quantile(quantile):
        return scipy.stats.norm.ppf(quantile)

    def update_scale_table(self, scale_table, force=False):
        """entropy_models.py:643-652."""
        if self._offset.numel() > 0 and not force:
            return False
        device = self.scale_table.device
        self.scale_table = self._prepare_scale_table(scale_table).to(device)
        self.update()
        return True

    @torch.no_grad()
    def update(self):
        """entropy_models.py:655-678 (without the reference's debug prints, :680-689)."""
        multiplier = -self._standardized_quantile(self.tail_mass / 2)
        pmf_center = torch.ceil(self.scale_table * multiplier).int()
        pmf_length = 2 * pmf_center + 1
        max_length = int(torch.max(pmf_length).item())
        device = pmf_center.device
        samples = torch.abs(torch.arange(max_length, device=device).int() - pmf_center[:, None]).float()
        samples_scale = self.scale_table.unsqueeze(1).float()
        upper = self._standardized_cumulative((0.5 - samples) / samples_scale)
        lower = self._standardized_cumulative((-0.5 - samples) / samples_scale)
        pmf = upper - lower
        tail_mass = 2 * lower[:, :1]
        self._quantized_cdf = self._pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
        self._offset = -pmf_center
        self._cdf_length = pmf_length + 2
