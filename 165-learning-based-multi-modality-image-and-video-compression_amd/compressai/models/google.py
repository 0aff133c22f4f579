"""Ballé 2018 / Minnen 2018 models (reference: compressai/models/google.py:58-692).

Same classes, constructor signatures (``channel`` argument of the fork
included), module names and state_dict keys.  Forward passes are the
reference's (google.py:172-182, 281-295, 379-391, 493-515) with two
MI355X-motivated differences that leave the arithmetic unchanged:
  * ``torch.abs(y)`` feeding h_a is applied inside the first h_a conv's
    operand load (and its backward sign mask inside that conv's dgrad);
  * conv -> ReLU/LeakyReLU pairs run fused (layers.Sequential);
and without the reference's debug prints (google.py:287-288).

The hyperprior models' forward can run the hyper branch (h_a, the
EntropyBottleneck, h_s, the GaussianConditional likelihood, and for the
context models the context / entropy-parameter stack) on a side stream while
g_s runs on the caller's stream: g_s only needs y_hat = y + noise, not the
scales.  The y noise is drawn once after z's (the reference's order) and
shared by y_hat and the likelihood; autograd runs each backward op on its
forward op's stream, so the backward overlaps the same way.  Outputs are the
reference's.  It is on by default for the context models only (measured on
MI355X, 50-step A/B x3: mbt2018 q1 B16 +2.6 %, cheng2020-anchor q6 B4 +0.7 %;
bmshj2018-hyperprior q1 B16 -0.8 %, mbt2018-mean -0.3 %: their hyper branch
is too short to hide anything and the second stream costs graph edges).
CAI_HYPER_STREAM=0/1 forces it off/on for every model.

compress / decompress (google.py:195-204, 325-344, 393-416, 526-692) follow
the reference: transforms on the HIP kernels (fp32 outside autocast, so the
encoder and decoder reproduce each other's scales exactly), symbols from the
quantize kernel, rANS strings from libcai_coder.so.  The autoregressive
models' serial per-latent-pixel loop runs the masked 5x5 context conv and
the 1x1 entropy-parameter stack on the same kernels, one pixel at a time.
"""
import math
import os
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..entropy_models import EntropyBottleneck, GaussianConditional
from ..entropy_models.entropy_models import _QuantizeFn, _draw_noise, _noise_for
from .._native import Q_DEQUANTIZE, Q_NOISE
from ..layers import GDN, MaskedConv2d, Sequential
from .._ops import CatFn, ChunkFn, ConvFn, ConvSpec, fan_out
from .._prepack import prepacked_forward
from ..ans import BufferedRansEncoder, RansDecoder
from ..layers.conv import Conv2d
from .utils import conv, deconv, update_registered_buffers

__all__ = ["CompressionModel", "FactorizedPrior", "ScaleHyperprior", "MeanScaleHyperprior",
           "JointAutoregressiveHierarchicalPriors", "get_scale_table", "SCALES_MIN", "SCALES_MAX", "SCALES_LEVELS"]

SCALES_MIN = 0.11
SCALES_MAX = 256
SCALES_LEVELS = 64


_HYPER_STREAM = os.environ.get("CAI_HYPER_STREAM", "auto")
_SIDE = {}


def _side_stream(t: torch.Tensor, default: bool):
    """The hyper branch's stream for t's device (None: run serially)."""
    on = default if _HYPER_STREAM == "auto" else _HYPER_STREAM == "1"
    if not on or not t.is_cuda:
        return None
    s = _SIDE.get(t.device)
    if s is None:
        s = _SIDE[t.device] = torch.cuda.Stream(device=t.device)
    return s


def _quantize_y(y, training):
    """y_hat = y + U(-1/2, 1/2) (training) / round(y) (eval): GaussianConditional.quantize without means.  The
    draw is made inside the quantize kernel (a DeviceDraw; the likelihood kernel on the side stream replays it)."""
    noise = _noise_for(y) if training else None
    return _QuantizeFn.apply(y, None, noise, Q_NOISE if training else Q_DEQUANTIZE), noise


def _z_noise(model, y):
    """z's training noise, drawn on the caller's stream BEFORE the hyper branch forks (the reference's draw
    order: z first, entropy_models.py:495-540 called from google.py:281-295): every draw of the step then
    runs on one stream, so the device generator's draw index and arrival ticket are never shared by two
    concurrent launches.  z = h_a(y) has the EntropyBottleneck's channels and two stride-2 halvings
    (k5 s2 p2 / k3 s2 p1: ceil(n / 2) each) of y's grid."""
    if not model.training:
        return None
    B, _, H, W = y.shape
    shape = (B, model.entropy_bottleneck.channels, -(-(-(-H // 2)) // 2), -(-(-(-W // 2)) // 2))
    return _draw_noise(torch.empty(shape, dtype=torch.float32, device=y.device, memory_format=torch.channels_last))


def _cross(main, side, y, noise, outs, z_noise=None):
    """Caching-allocator bookkeeping of the tensors that cross between the two streams."""
    y.record_stream(side)
    if z_noise is not None:
        z_noise.record_stream(side)
    if noise is not None:
        noise.record_stream(side)
    for t in outs:
        t.record_stream(main)


# ScaleHyperprior: h_s's trailing ReLU masked in the GaussianConditional's backward (CAI_GC_RELU=0: by the conv's
# own act-backward launch, A/B)
_GC_RELU = os.environ.get("CAI_GC_RELU", "1") == "1"


def get_scale_table(min=SCALES_MIN, max=SCALES_MAX, levels=SCALES_LEVELS):
    return torch.exp(torch.linspace(math.log(min), math.log(max), levels))


class CompressionModel(nn.Module):
    # data parallelism (compressai.distributed.OverlappedAllReduce): the parameters upstream of the cut the
    # forward marks with _dp_cut (name prefixes) form the tail; dp_tail_cuts (children of the tail Sequential,
    # outermost first) cut it further at their inputs, one gradient bucket per piece, each all-reduced while
    # the pieces below it run their backward.  _analysis: g_a[4:], g_a[2:4], g_a[:2] (the last, exposed one
    # is conv(3, N) + GDN: 26 K parameters at N = 128)
    dp_tail = ("g_a.",)
    dp_tail_cuts = ("g_a.4", "g_a.2")
    # dp_phases(): the head split too -- g_s first (its gradients are final first: the loss reaches x_hat
    # before anything else), in pieces at the inputs of dp_gs_cuts (children of g_s, outermost first), then the
    # entropy path: dp_head_splits, each (param prefixes, the cut it stops at besides y), then what is left
    dp_split_head = False     # the forward marks gs_in / the likelihoods (google.py, waseda.py models)
    dp_gs_cuts = ()
    dp_head_splits = ()
    _dp_cut_fn = None
    _dp_mark_fn = None

    def _dp_mark(self, name, *ts):
        """Identity, unless a bucketed exchange is attached (compressai.distributed.OverlappedAllReduce): then
        boundary nodes at this named point of the graph (a cut of its phase plan)."""
        if self._dp_mark_fn is not None:
            ts = self._dp_mark_fn(name, *ts)
        return ts[0] if len(ts) == 1 else ts

    def _dp_cut(self, *ts):
        """The cut between the head and the tail (dp_tail): y = g_a(x) for the zoo models."""
        if self._dp_cut_fn is not None:      # an exchange built from dp_tail / dp_tail_cuts alone
            ts = self._dp_cut_fn(*ts)
            return ts[0] if len(ts) == 1 else ts
        return self._dp_mark("y", *ts)

    # the cuts the synthesis / entropy path marks in forward (dp_phases): g_s's input, each likelihood tensor
    _dp_synth = "g_s"
    _dp_synth_in = "gs_in"
    _dp_liks = ("lik_y", "lik_z")

    def dp_phases(self):
        """The bucketed gradient exchange's backward phases, in backward order (compressai.distributed,
        configure_optimizers(phases=...)): (parameter-name prefixes of the phase's bucket (None: all the rest),
        root cuts, input cuts).  Synthesis pieces first, then the entropy path (dp_head_splits), then the tail
        (dp_tail) in the pieces dp_tail_cuts makes."""
        from ..optim import check_tail_cuts

        if not self.dp_split_head:      # a forward that marks only y: one head bucket
            return [(None, ["loss"], ["y"])] + self._dp_tail_phases()
        syn = self._dp_synth
        gs_cuts = check_tail_cuts(self.dp_gs_cuts)
        liks = list(self._dp_liks)
        ph = []
        prev, hi = ["loss"], len(self.get_submodule(syn))
        for c in gs_cuts:                                   # g_s[k:] pieces, outermost first
            k = int(c.rsplit(".", 1)[1])
            ph.append(([f"{syn}.{j}." for j in range(k, hi)], prev, [c] + (liks if prev == ["loss"] else [])))
            prev, hi = [c], k
        ph.append(([f"{syn}.{j}." for j in range(hi)], prev,
                   [self._dp_synth_in] + (liks if prev == ["loss"] else [])))
        roots = [self._dp_synth_in] + liks[:1]
        pending = liks[1:]
        for prefixes, cut in self.dp_head_splits:           # e.g. the context / entropy-parameter stack
            # it stops at its cut AND at "yq" -- y as its other consumers (quantize, GaussianConditional)
            # read it -- not at y itself: the hyper path below the cut also leads to y, and an input reachable
            # from another input of one phase would pull that path into the phase
            ph.append((list(prefixes), roots, [cut, "yq"]))
            roots = [cut] + pending
            pending = []
        ph.append((None, roots + pending, ["y"]))           # the rest of the head
        return ph + self._dp_tail_phases(["y", "yq"] if self.dp_head_splits else ["y"])

    def _dp_tail_phases(self, first_roots=("y",)):
        """The tail (dp_tail) in the pieces dp_tail_cuts makes, from y (and the cuts still holding y's other
        gradients) down to the input."""
        from ..optim import check_tail_cuts

        ph = []
        tail_cuts = check_tail_cuts(self.dp_tail_cuts)
        prev = list(first_roots)
        parent = None
        hi = None
        for c in tail_cuts:
            parent, idx = c.rsplit(".", 1)
            hi = len(self.get_submodule(parent)) if hi is None else hi
            ph.append(([f"{parent}.{j}." for j in range(int(idx), hi)], prev, [c]))
            prev, hi = [c], int(idx)
        last = [f"{parent}.{j}." for j in range(hi)] if tail_cuts else list(self.dp_tail)
        ph.append((last, prev, []))
        return ph

    def __init__(self, entropy_bottleneck_channels, init_weights=None):
        super().__init__()
        self.entropy_bottleneck = EntropyBottleneck(entropy_bottleneck_channels)
        if init_weights is not None:
            warnings.warn("init_weights was removed as it was never functional", DeprecationWarning)

    def aux_loss(self):
        # the reference's sum(...) (google.py:79-86) without its int 0 start value: 0 + loss is one more
        # device launch per step; the same value (a lone module's loss itself)
        losses = [m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck)]
        if not losses:
            return 0
        total = losses[0]
        for extra in losses[1:]:
            total = total + extra
        return total

    def forward(self, *args):
        raise NotImplementedError()

    def __call__(self, *args, **kwargs):
        if getattr(self, "_is_replica", False):
            # nn.DataParallel (the reference's CustomDataParallel, examples/train.py:101-108,422-423, taken when
            # torch.cuda.device_count() > 1) runs replicas in one host thread per GPU over broadcast weight copies;
            # this build scales one process per GPU instead (compressai.distributed over RCCL)
            raise RuntimeError(
                f"{type(self).__name__}: nn.DataParallel replicas are not supported by the MI355X build; run one "
                "process per GPU (torchrun --nproc-per-node N, gradients exchanged by compressai.distributed: "
                "OverlappedAllReduce / allreduce_mean_), or make one GPU visible (HIP_VISIBLE_DEVICES=0) so the "
                "training script does not wrap the model")
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
    # gradient buckets (dp_phases): g_s, the EntropyBottleneck, then g_a in pieces
    dp_split_head = True
    _dp_liks = ("lik_y",)
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
        y = self._dp_cut(self.g_a(x))
        y_hat, y_likelihoods = self.entropy_bottleneck(y)
        x_hat = self.g_s(self._dp_mark("gs_in", y_hat))
        return {"x_hat": x_hat, "likelihoods": {"y": self._dp_mark("lik_y", y_likelihoods)}}

    @classmethod
    def from_state_dict(cls, state_dict, channel=3):
        net = cls(state_dict["g_a.0.weight"].size(0), state_dict["g_a.6.weight"].size(0), channel=channel)
        net.load_state_dict(state_dict)
        return net

    @torch.no_grad()
    def compress(self, x):
        """google.py:195-198."""
        with prepacked_forward(self):
            y = self.g_a(x)
            y_strings = self.entropy_bottleneck.compress(y)
        return {"strings": [y_strings], "shape": y.size()[-2:]}

    @torch.no_grad()
    def decompress(self, strings, shape):
        """google.py:200-204."""
        assert isinstance(strings, list) and len(strings) == 1
        with prepacked_forward(self):
            y_hat = self.entropy_bottleneck.decompress(strings[0], shape)
            x_hat = self.g_s(y_hat).clamp_(0, 1)
        return {"x_hat": x_hat}


class ScaleHyperprior(CompressionModel):
    # gradient buckets (dp_phases): g_s, the hyper path (h_a, h_s, EntropyBottleneck), then g_a in pieces
    dp_split_head = True
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
        y = self._dp_cut(self.g_a(x))
        side = _side_stream(y, False)
        if side is None:
            y_ha, y_gc = fan_out(y)                  # y's two gradients meet in h_a's first dgrad epilogue
            z = self.h_a(y_ha, input_abs=True)       # h_a(|y|)
            z_hat, z_likelihoods = self.entropy_bottleneck(z)
            # h_s's trailing ReLU: its backward mask applied by the GaussianConditional's backward
            scales_hat = self.h_s(z_hat, act_bwd_downstream=_GC_RELU)
            y_hat, y_likelihoods = self.gaussian_conditional(y_gc, scales_hat, scales_relu=_GC_RELU)
            x_hat = self.g_s(self._dp_mark("gs_in", y_hat))
            return {"x_hat": x_hat, "likelihoods": {"y": self._dp_mark("lik_y", y_likelihoods),
                                                    "z": self._dp_mark("lik_z", z_likelihoods)}}
        main = torch.cuda.current_stream()
        z_noise = _z_noise(self, y)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            z = self.h_a(y, input_abs=True)
            z_hat, z_likelihoods = self.entropy_bottleneck(z, noise=z_noise)
            scales_hat = self.h_s(z_hat, act_bwd_downstream=_GC_RELU)
        y_hat, noise = _quantize_y(y, self.training)
        ready = torch.cuda.Event()
        ready.record(main)
        x_hat = self.g_s(self._dp_mark("gs_in", y_hat))
        with torch.cuda.stream(side):
            side.wait_event(ready)
            _, y_likelihoods = self.gaussian_conditional(y, scales_hat, noise=noise, scales_relu=_GC_RELU)
        main.wait_stream(side)
        _cross(main, side, y, noise, (z_likelihoods, y_likelihoods), z_noise)
        return {"x_hat": x_hat, "likelihoods": {"y": self._dp_mark("lik_y", y_likelihoods),
                                                "z": self._dp_mark("lik_z", z_likelihoods)}}

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

    @torch.no_grad()
    def compress(self, x):
        """google.py:325-335."""
        with prepacked_forward(self):
            y = self.g_a(x)
            z = self.h_a(y, input_abs=True)
            z_strings = self.entropy_bottleneck.compress(z)
            z_hat = self.entropy_bottleneck.decompress(z_strings, z.size()[-2:])
            scales_hat = self.h_s(z_hat)
            indexes = self.gaussian_conditional.build_indexes(scales_hat)
            y_strings = self.gaussian_conditional.compress(y, indexes)
        return {"strings": [y_strings, z_strings], "shape": z.size()[-2:]}

    @torch.no_grad()
    def decompress(self, strings, shape):
        """google.py:337-344."""
        assert isinstance(strings, list) and len(strings) == 2
        with prepacked_forward(self):
            z_hat = self.entropy_bottleneck.decompress(strings[1], shape)
            scales_hat = self.h_s(z_hat)
            indexes = self.gaussian_conditional.build_indexes(scales_hat)
            y_hat = self.gaussian_conditional.decompress(strings[0], indexes, z_hat.dtype)
            x_hat = self.g_s(y_hat).clamp_(0, 1)
        return {"x_hat": x_hat}


class MeanScaleHyperprior(ScaleHyperprior):
    def __init__(self, N, M, channel=3, **kwargs):
        super().__init__(N, M, channel, **kwargs)
        self.h_a = Sequential(conv(M, N, stride=1, kernel_size=3), nn.LeakyReLU(inplace=True),
                              conv(N, N), nn.LeakyReLU(inplace=True), conv(N, N))
        self.h_s = Sequential(deconv(N, M), nn.LeakyReLU(inplace=True), deconv(M, M * 3 // 2),
                              nn.LeakyReLU(inplace=True), conv(M * 3 // 2, M * 2, stride=1, kernel_size=3))

    def forward(self, x):
        y = self._dp_cut(self.g_a(x))
        side = _side_stream(y, False) if self.training else None   # eval: y_hat = round(y - means) + means
        if side is None:
            y_ha, y_gc = fan_out(y)
            z = self.h_a(y_ha)
            z_hat, z_likelihoods = self.entropy_bottleneck(z)
            scales_hat, means_hat = ChunkFn.apply(self.h_s(z_hat))
            y_hat, y_likelihoods = self.gaussian_conditional(y_gc, scales_hat, means=means_hat)
            x_hat = self.g_s(self._dp_mark("gs_in", y_hat))
            return {"x_hat": x_hat, "likelihoods": {"y": self._dp_mark("lik_y", y_likelihoods),
                                                    "z": self._dp_mark("lik_z", z_likelihoods)}}
        main = torch.cuda.current_stream()
        z_noise = _z_noise(self, y)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            z = self.h_a(y)
            z_hat, z_likelihoods = self.entropy_bottleneck(z, noise=z_noise)
            scales_hat, means_hat = ChunkFn.apply(self.h_s(z_hat))
        y_hat, noise = _quantize_y(y, True)         # noise mode ignores the means
        ready = torch.cuda.Event()
        ready.record(main)
        x_hat = self.g_s(self._dp_mark("gs_in", y_hat))
        with torch.cuda.stream(side):
            side.wait_event(ready)
            _, y_likelihoods = self.gaussian_conditional(y, scales_hat, means=means_hat, noise=noise)
        main.wait_stream(side)
        _cross(main, side, y, noise, (z_likelihoods, y_likelihoods), z_noise)
        return {"x_hat": x_hat, "likelihoods": {"y": self._dp_mark("lik_y", y_likelihoods),
                                                "z": self._dp_mark("lik_z", z_likelihoods)}}

    @torch.no_grad()
    def compress(self, x):
        """google.py:393-404."""
        with prepacked_forward(self):
            y = self.g_a(x)
            z = self.h_a(y)
            z_strings = self.entropy_bottleneck.compress(z)
            z_hat = self.entropy_bottleneck.decompress(z_strings, z.size()[-2:])
            scales_hat, means_hat = ChunkFn.apply(self.h_s(z_hat))
            indexes = self.gaussian_conditional.build_indexes(scales_hat)
            y_strings = self.gaussian_conditional.compress(y, indexes, means=means_hat)
        return {"strings": [y_strings, z_strings], "shape": z.size()[-2:]}

    @torch.no_grad()
    def decompress(self, strings, shape):
        """google.py:406-416."""
        assert isinstance(strings, list) and len(strings) == 2
        with prepacked_forward(self):
            z_hat = self.entropy_bottleneck.decompress(strings[1], shape)
            scales_hat, means_hat = ChunkFn.apply(self.h_s(z_hat))
            indexes = self.gaussian_conditional.build_indexes(scales_hat)
            y_hat = self.gaussian_conditional.decompress(strings[0], indexes, means=means_hat)
            x_hat = self.g_s(y_hat).clamp_(0, 1)
        return {"x_hat": x_hat}


class _ARCoding:
    """Serial autoregressive entropy coding of the context models (google.py:565-608, 654-692), shared by
    JointAutoregressiveHierarchicalPriors and the multi-modal Guided / Master codecs (master.py:993-1147,
    1337-1464): per latent pixel, the masked 5x5 context conv (valid, on a crop) and the 1x1
    entropy-parameter stack run on the HIP kernels, fp32, so encoder and decoder agree exactly."""

    _AR_SPEC = None

    def _ar_params(self, y_crop, p):
        """Entropy parameters of the centre pixel of a 5x5 crop: masked context conv
        (valid, no padding) + the 1x1 stack (google.py:580-592 / 671-681)."""
        if _ARCoding._AR_SPEC is None:
            _ARCoding._AR_SPEC = ConvSpec(5, 1, 0)
        cp = self.context_prediction
        ctx_p = ConvFn.apply(y_crop, cp.weight, cp.bias, _ARCoding._AR_SPEC)
        return ChunkFn.apply(self.entropy_parameters(CatFn.apply(p, ctx_p)))

    def _gc_tables(self):
        gc = self.gaussian_conditional
        return gc._quantized_cdf.tolist(), gc._cdf_length.tolist(), gc._offset.tolist()

    @staticmethod
    def _warn_gpu(model):
        if next(model.parameters()).device != torch.device("cpu"):
            warnings.warn("Inference on GPU is not recommended for the autoregressive models (the entropy coder is "
                          "run sequentially on CPU).")

    def _ar_encode_all(self, y, params):
        """y_strings of a batch (google.py:542-561)."""
        cp = self.context_prediction
        cp.weight.data *= cp.mask          # MaskedConv2d semantics (layers.py:75-78)
        kernel_size = 5
        padding = (kernel_size - 1) // 2
        y_height, y_width = params.size(2), params.size(3)
        y_hat = F.pad(y.float(), (padding, padding, padding, padding))
        return [self._compress_ar(y_hat[i:i + 1], params[i:i + 1], y_height, y_width, kernel_size, padding)
                for i in range(y.size(0))]

    def _ar_decode_all(self, y_strings, params):
        """y_hat of a batch (google.py:622-650)."""
        cp = self.context_prediction
        cp.weight.data *= cp.mask
        kernel_size = 5
        padding = (kernel_size - 1) // 2
        y_height, y_width = params.size(2), params.size(3)
        y_hat = torch.zeros((params.size(0), self.M, y_height + 2 * padding, y_width + 2 * padding),
                            device=params.device)
        for i, y_string in enumerate(y_strings):
            self._decompress_ar(y_string, y_hat[i:i + 1], params[i:i + 1], y_height, y_width, kernel_size, padding)
        return F.pad(y_hat, (-padding, -padding, -padding, -padding))

    def _compress_ar(self, y_hat, params, height, width, kernel_size, padding):
        """google.py:565-608."""
        cdf, cdf_lengths, offsets = self._gc_tables()
        encoder = BufferedRansEncoder()
        symbols_list, indexes_list = [], []
        gc = self.gaussian_conditional
        for h in range(height):
            for w in range(width):
                y_crop = y_hat[:, :, h:h + kernel_size, w:w + kernel_size]
                p = params[:, :, h:h + 1, w:w + 1]
                scales_hat, means_hat = self._ar_params(y_crop, p)
                indexes = gc.build_indexes(scales_hat)
                y_c = y_crop[:, :, padding:padding + 1, padding:padding + 1]
                y_q = gc.quantize(y_c, "symbols", means_hat)
                y_hat[:, :, h + padding:h + padding + 1, w + padding:w + padding + 1] = y_q.float() + means_hat.float()
                symbols_list.extend(y_q.reshape(-1).tolist())
                indexes_list.extend(indexes.reshape(-1).tolist())
        encoder.encode_with_indexes(symbols_list, indexes_list, cdf, cdf_lengths, offsets)
        return encoder.flush()

    def _decompress_ar(self, y_string, y_hat, params, height, width, kernel_size, padding):
        """google.py:654-692."""
        cdf, cdf_lengths, offsets = self._gc_tables()
        decoder = RansDecoder()
        decoder.set_stream(y_string)
        gc = self.gaussian_conditional
        for h in range(height):
            for w in range(width):
                y_crop = y_hat[:, :, h:h + kernel_size, w:w + kernel_size]
                p = params[:, :, h:h + 1, w:w + 1]
                scales_hat, means_hat = self._ar_params(y_crop, p)
                indexes = gc.build_indexes(scales_hat)
                rv = decoder.decode_stream(indexes.reshape(-1).tolist(), cdf, cdf_lengths, offsets)
                rv = torch.tensor(rv, dtype=torch.float32, device=y_hat.device).reshape(1, -1, 1, 1)
                rv = gc.dequantize(rv, means_hat.float())
                y_hat[:, :, h + padding:h + padding + 1, w + padding:w + padding + 1] = rv


class JointAutoregressiveHierarchicalPriors(_ARCoding, MeanScaleHyperprior):
    # gradient buckets (dp_phases): g_s (pieces: dp_gs_cuts), the context model + entropy parameters (their
    # gradients are final once the backward reaches h_s's output, cut "params"), the hyper path, then g_a
    dp_head_splits = ((("entropy_parameters.", "context_prediction."), "params"),)
    def __init__(self, N=192, M=192, channel=3, **kwargs):
        super().__init__(N=N, M=M, channel=channel, **kwargs)
        self.entropy_parameters = Sequential(
            Conv2d(M * 12 // 3, M * 10 // 3, 1), nn.LeakyReLU(inplace=True),
            Conv2d(M * 10 // 3, M * 8 // 3, 1), nn.LeakyReLU(inplace=True),
            Conv2d(M * 8 // 3, M * 6 // 3, 1))
        self.context_prediction = MaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)

    def forward(self, x):
        y = self._dp_cut(self.g_a(x))
        side = _side_stream(y, True)
        if side is None:
            y_ha, y_q, y_gc = fan_out(y, 3, absorb=False)
            y_q, y_gc = self._dp_mark("yq", y_q, y_gc)   # y as quantize / the GaussianConditional read it
            z = self.h_a(y_ha)
            z_hat, z_likelihoods = self.entropy_bottleneck(z)
            params = self._dp_mark("params", self.h_s(z_hat))
            y_hat = self.gaussian_conditional.quantize(y_q, "noise" if self.training else "dequantize")
            y_ctx, y_gs = fan_out(y_hat, absorb=False)
            ctx_params = self.context_prediction(y_ctx)
            gaussian_params = self.entropy_parameters(CatFn.apply(params, ctx_params))
            scales_hat, means_hat = ChunkFn.apply(gaussian_params)
            _, y_likelihoods = self.gaussian_conditional(y_gc, scales_hat, means=means_hat)
            x_hat = self.g_s(self._dp_mark("gs_in", y_gs))
            return {"x_hat": x_hat, "likelihoods": {"y": self._dp_mark("lik_y", y_likelihoods),
                                                    "z": self._dp_mark("lik_z", z_likelihoods)}}
        main = torch.cuda.current_stream()
        z_noise = _z_noise(self, y)
        y_ha, y_q, y_gc = fan_out(y, 3, absorb=False)   # y's three gradients: native adds, not ATen's
        y_q, y_gc = self._dp_mark("yq", y_q, y_gc)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            z = self.h_a(y_ha)
            z_hat, z_likelihoods = self.entropy_bottleneck(z, noise=z_noise)
            params = self._dp_mark("params", self.h_s(z_hat))
        # the reference's draws in its order (z, then y_hat's, then the likelihood's)
        y_hat, noise = _quantize_y(y_q, self.training)
        noise2 = _draw_noise(y) if self.training else None
        y_gs, y_ctx = fan_out(y_hat, absorb=False)
        ready = torch.cuda.Event()
        ready.record(main)
        x_hat = self.g_s(self._dp_mark("gs_in", y_gs))
        with torch.cuda.stream(side):
            side.wait_event(ready)
            ctx_params = self.context_prediction(y_ctx)
            gaussian_params = self.entropy_parameters(CatFn.apply(params, ctx_params))
            scales_hat, means_hat = ChunkFn.apply(gaussian_params)
            _, y_likelihoods = self.gaussian_conditional(y_gc, scales_hat, means=means_hat, noise=noise2)
        main.wait_stream(side)
        y_hat.record_stream(side)
        if noise2 is not None:
            noise2.record_stream(side)
        _cross(main, side, y, noise, (z_likelihoods, y_likelihoods), z_noise)
        return {"x_hat": x_hat, "likelihoods": {"y": self._dp_mark("lik_y", y_likelihoods),
                                                "z": self._dp_mark("lik_z", z_likelihoods)}}

    @torch.no_grad()
    def compress(self, x):
        """google.py:526-563."""
        self._warn_gpu(self)
        with prepacked_forward(self):
            y = self.g_a(x)
            z = self.h_a(y)
            z_strings = self.entropy_bottleneck.compress(z)
            z_hat = self.entropy_bottleneck.decompress(z_strings, z.size()[-2:])
            params = self.h_s(z_hat)
            y_strings = self._ar_encode_all(y, params)
        return {"strings": [y_strings, z_strings], "shape": z.size()[-2:]}

    @torch.no_grad()
    def decompress(self, strings, shape):
        """google.py:610-652."""
        assert isinstance(strings, list) and len(strings) == 2
        self._warn_gpu(self)
        with prepacked_forward(self):
            z_hat = self.entropy_bottleneck.decompress(strings[1], shape)
            params = self.h_s(z_hat)
            y_hat = self._ar_decode_all(strings[0], params)
            x_hat = self.g_s(y_hat).clamp_(0, 1)
        return {"x_hat": x_hat}
