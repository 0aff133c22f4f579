"""Autograd functions over libcai (HIP kernels for gfx950).

Tensor convention: activations travel between these functions as
*pixel-major* tensors -- logical NCHW ``[B, C, H, W]`` with
``torch.channels_last`` strides (element (p, c) at ``p*ld + c``).  A channel
slice of a wider pixel-major tensor (``chunk(2, 1)``) is pixel-major with
``ld > C`` and is consumed without a copy.

Compute precision: inside ``torch.autocast("cuda")`` the conv / GDN operands
are bf16 (fp32 MFMA accumulation) -- the counterpart of the reference's
``torch.cuda.amp.autocast`` training (examples/train.py:172-173); outside it
everything runs in exact fp32 (v_mfma_f32_16x16x4_f32), which is the mode the
parity tests compare against the CPU oracle.  Likelihoods and losses are
always fp32.

Every op here launches HIP kernels on ``torch.cuda.current_stream()``; CPU
tensors are rejected (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes
import math
import os
import warnings
from typing import Optional, Sequence, Tuple

import torch

from . import _ledger
from ._native import (ACT_LEAKY, ACT_NONE, ACT_RELU, BF16, F32, MASK_BEFORE_RES, MASK_LEAKY, MASK_NONE, MASK_POS,
                      Q_DEQUANTIZE, Q_NOISE,
                      GC_SCALES_RELU, JOB_EDGE, JOB_GDN, JOB_NONE, JOB_WGRAD, NOISE_BUF, NOISE_DRAW, NOISE_REPLAY, ConvGeom, EbGrads, EbParams, NoiseSrc, RdGrads,
                      RdInputs, ReduceJob, ResunitArgs, ResunitWgradArgs, WgradCall, lib)

_VP = ctypes.c_void_p
_GDN_TWO_PASS = os.environ.get("CAI_GDN_TWO_PASS", "0") == "1"   # A/B knobs (tools/ab_env.sh)
_RD_UNFUSED = os.environ.get("CAI_RD_UNFUSED", "0") == "1"
_EDGE_OFF = os.environ.get("CAI_EDGE_OFF", "0") == "1"


# ---------------------------------------------------------------------------
# small helpers
# ---------------------------------------------------------------------------

DIRECT_GRAD_ATTR = "_cai_direct_grad"


def direct_grad(p) -> bool:
    """True when p.grad is a live fp32 view the kernels may accumulate into (set by optim.FusedAdam)."""
    return (p is not None and getattr(p, DIRECT_GRAD_ATTR, False) and p.grad is not None
            and p.grad.dtype == torch.float32 and p.grad.is_contiguous())


def _es(dtype) -> int:
    return 2 if dtype == torch.bfloat16 else 4


def _conv_kernel(g, dt, direction, in_abs=0):
    return lambda: lib.cai_conv_kernel_name(ctypes.byref(g), dcode(dt), direction, int(in_abs)).decode()


def _stream() -> _VP:
    return _VP(torch.cuda.current_stream().cuda_stream)


# ---------------------------------------------------------------------------
# weight gradients on a side stream
# ---------------------------------------------------------------------------
# A conv's weight gradient feeds nothing but the optimizer, so when it lands straight in the optimizer's flat
# buffer (direct_grad) it is launched on a per-device side stream: the input-gradient chain -- the backward's
# critical path -- goes on without it, and inside a captured graph the two become parallel branches on two
# hardware queues.  The side stream joins the caller's stream in an autograd final callback (as
# DistributedDataParallel finalises its buckets), i.e. before backward() returns, so .grad reads after
# backward see the finished values.  Off by default (CAI_WGRAD_STREAM=1 turns it on): measured on MI355X,
# 50-step A/B x2, it costs 1.5-3.5 % on bmshj2018-hyperprior q1/q6 and mbt2018 (cheng2020-anchor even) --
# the captured graph's cross-queue edges cost more than the overlap returns (profiles/r02_wgrad_stream_ab.log).
# The per-launch ledger always runs in-stream.
_WGRAD_STREAM = os.environ.get("CAI_WGRAD_STREAM", "0") == "1"
_WSIDE = {}
_WPENDING = set()


def _join_wgrad(device):
    _WPENDING.discard(device)
    torch.cuda.current_stream(device).wait_stream(_WSIDE[device])


class _WgradLaunch:
    """Context for one direct weight-gradient launch: on the side stream (after the current stream's work
    so far), with the inputs' memory kept alive for it; None-valued side when not applicable."""

    def __init__(self, device, direct: bool, *inputs):
        self.side = None
        if not (_WGRAD_STREAM and direct and _ledger.active() is None):
            return
        side = _WSIDE.get(device)
        if side is None:
            side = _WSIDE[device] = torch.cuda.Stream(device=device)
        self.side, self.inputs = side, inputs

    def __enter__(self):
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream(self.side.device))
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.side is None:
            return False
        self._ctx.__exit__(*exc)
        for t in self.inputs:
            if t is not None:
                t.record_stream(self.side)
        dev = self.side.device
        if dev not in _WPENDING:
            _WPENDING.add(dev)
            torch.autograd.Variable._execution_engine.queue_callback(lambda: _join_wgrad(dev))
        return False


# Deferred weight-gradient partial kernels of SMALL layers (<= CAI_WGRAD_SIDE_PX G pixels) on the side stream: they
# touch only their slabs until the deferred reduce (which waits for the side stream), so they can run under the
# input-gradient chain; 0 = off.
_WGRAD_SIDE_PX = int(os.environ.get("CAI_WGRAD_SIDE_PX", "0"))


class _SideDeferred:
    def __init__(self, device, npix: int, *inputs):
        self.side = None
        if not (_WGRAD_SIDE_PX and npix <= _WGRAD_SIDE_PX and _ledger.active() is None):
            return
        side = _WSIDE.get(device)
        if side is None:
            side = _WSIDE[device] = torch.cuda.Stream(device=device)
        self.side, self.inputs = side, inputs

    def __enter__(self):
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream(self.side.device))
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.side is not None:
            self._ctx.__exit__(*exc)
            for t in self.inputs:
                if t is not None:
                    t.record_stream(self.side)
        return False


# ---------------------------------------------------------------------------
# deferred parameter-gradient reduces (cai_reduce_jobs, csrc/reduce_jobs.hip)
# ---------------------------------------------------------------------------
# The weight gradients that land straight in the optimizer's flat buffer (direct_grad) are read by nothing
# before the optimizer, so their final fixed-order reduces (conv weight-gradient slabs, fused-GDN partials)
# are queued per stream during the backward pass and run in ONE launch (per 32 jobs) from an autograd final
# callback -- before backward() returns, so .grad reads after backward see the finished values -- instead of
# one launch after every layer.  The job's workspace is kept alive until that launch.  Bit-identical to the
# immediate path (same kernel).  Off under the per-launch ledger (it replays single calls) and when a weight
# gradient runs on the side stream.  CAI_DEFER_REDUCE=0 turns it off (A/B).
_DEFER_REDUCE = os.environ.get("CAI_DEFER_REDUCE", "1") == "1"
_REDUCE_SPLIT = os.environ.get("CAI_REDUCE_SPLIT", "0") == "1"   # diagnostics: one launch per deferred job
_JOBS = {}          # (device, graph task id) -> [jobs, streams, keep-alive tensors, wgrad calls, device, unit calls,
                    #                            early-reduce stream, bytes queued since the last early reduce]
# The latent layers' weight gradients (wgrad_small_kernel: <= 1024 G pixels) are deferred the same way, as whole
# calls: the flush runs them in one launch (cai_conv_wgrad_batch) ahead of the reduce launch, instead of one
# launch per layer in the backward's chain; so are the ResidualUnits' weight gradients (cai_resunit_wgrad_batch: one
# launch for a backward's units).  CAI_WGRAD_BATCH=0 launches both in place (A/B).
_WGRAD_BATCH = os.environ.get("CAI_WGRAD_BATCH", "1") == "1"
# Early reduces: once the queued jobs' partials pass CAI_EARLY_REDUCE_MB, they are reduced on a per-device side
# stream (forked from the backward's stream after their partial kernels) while the backward goes on -- the
# loss-side layers' slabs (C2: g_s's weight-gradient slabs and GDN partials, ~150 MB) under the latent chain's
# small launches -- and the final flush joins that stream before its own launch.  Safe because a gradient with a
# deferred job has no immediate writer in the same backward (every direct-grad path defers); two jobs that write
# one gradient stay ordered (the side stream's launches in queue order, the final flush after the join).  0 = off.
_EARLY_BYTES = float(os.environ.get("CAI_EARLY_REDUCE_MB", "0")) * 1e6
_EARLY_BLOCKS = int(os.environ.get("CAI_EARLY_REDUCE_BLOCKS", "0"))   # grid cap of the early launches (0: none)
_EARLY_MAX = int(os.environ.get("CAI_EARLY_REDUCE_MAX", "1"))          # early launches per backward
_RSIDE = {}


def _job_bytes(j) -> float:
    """Partial bytes a reduce job reads (its slab / per-block partials)."""
    if j.kind == JOB_WGRAD:
        return 4.0 * j.i[0] * j.i[1] * j.i[2]
    if j.kind == JOB_GDN:
        return 4.0 * j.i[0] * (j.i[1] * j.i[1] + j.i[1])
    if j.kind == JOB_EDGE:
        return 4.0 * j.i[1] * (9 * 16 * j.i[0] + 16)
    return 0.0


def _early_flush(pend):
    """Reduce the jobs queued so far on the side stream (after every stream their partial kernels ran on)."""
    dev = pend[4]
    side = _RSIDE.get(dev)
    if side is None:
        side = _RSIDE[dev] = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)
    for s in {s.cuda_stream: s for s in pend[1]}.values():
        if s.cuda_stream != cur.cuda_stream:
            side.wait_stream(s)
    jobs = pend[0]
    arr = (ReduceJob * len(jobs))(*jobs)
    lib.cai_reduce_jobs_grid(arr, len(jobs), _EARLY_BLOCKS, _VP(side.cuda_stream))
    for t in pend[2]:
        t.record_stream(side)
    pend[0] = []
    pend[6] = side
    pend[7] = 0.0


def _flush_jobs(key):
    """Run the jobs queued under `key` = (device, graph task) on the current stream (the backward caller's, as
    DDP's finalize uses it), after it has waited for every other stream a job's partial kernel ran on (the
    hyper branch's side stream: inside a captured graph this is the join edge)."""
    pend = _JOBS.pop(key, None)
    if not pend:
        return
    dev = key[0]
    cur = torch.cuda.current_stream(dev)
    if pend[6] is not None:
        cur.wait_stream(pend[6])        # join the early reduces
    if not (pend[0] or pend[3] or pend[5]):
        return
    jobs, streams, keep, calls = pend[:4]
    for s in {s.cuda_stream: s for s in streams}.values():
        if s.cuda_stream != cur.cuda_stream:
            cur.wait_stream(s)
    if calls:
        arr = (WgradCall * len(calls))(*calls)
        out = (ReduceJob * len(calls))()
        lib.cai_conv_wgrad_batch(arr, len(calls), _VP(cur.cuda_stream), out)
        jobs = jobs + [j for j in out if j.kind != JOB_NONE]
    units = pend[5]
    if units:
        args = (ResunitWgradArgs * len(units))(*[u[0] for u in units])
        wss = (ctypes.c_void_p * len(units))(*[u[1] for u in units])
        nbs = (ctypes.c_size_t * len(units))(*[u[2] for u in units])
        out = (ReduceJob * (3 * len(units)))()
        lib.cai_resunit_wgrad_batch(args, wss, nbs, len(units), _VP(cur.cuda_stream), out)
        jobs = jobs + [j for j in out if j.kind != JOB_NONE]
    if not jobs:
        for t in keep:
            t.record_stream(cur)
        return
    if _REDUCE_SPLIT:   # diagnostics: one launch per job (per-job times in a kernel trace)
        for j in jobs:
            one = (ReduceJob * 1)(j)
            lib.cai_reduce_jobs(one, 1, _VP(cur.cuda_stream))
    else:
        arr = (ReduceJob * len(jobs))(*jobs)
        lib.cai_reduce_jobs(arr, len(jobs), _VP(cur.cuda_stream))
    for t in keep:
        t.record_stream(cur)    # the caching allocator frees them for reuse only after these launches


def defer_reduce_ok(direct: bool) -> bool:
    """Deferred only inside a running backward (its final callback runs the jobs)."""
    return (_DEFER_REDUCE and direct and _ledger.active() is None and not _WGRAD_STREAM
            and torch._C._current_graph_task_id() >= 0)


def defer_job(job: "ReduceJob", device: torch.device, *keep: torch.Tensor):
    """Queue `job` (filled by a cai_*_deferred call on the current stream) until the end of this backward.

    The queue is keyed on the running graph task, so concurrent backwards (one host thread per replica) keep
    their own queues and each backward registers its own final callback: a backward that raised before its
    callback ran leaves only its own (never-run) entry behind, not a queue that later backwards would join
    without a flush.  Two jobs writing the same gradient (a module called twice in one forward) run in
    separate launches, in queue order (csrc/reduce_jobs.hip launch_reduce_jobs)."""
    if job.kind == JOB_NONE:
        return
    pend = _pending(device)
    pend[0].append(job)
    pend[1].append(torch.cuda.current_stream(pend[4]))
    pend[2].extend(t for t in keep if t is not None)
    if _EARLY_BYTES > 0 and pend[8] < _EARLY_MAX:
        pend[7] += _job_bytes(job)
        if pend[7] >= _EARLY_BYTES:
            _early_flush(pend)
            pend[8] += 1


def _pending(device: torch.device):
    dev = device.index if device.index is not None else torch.cuda.current_device()
    key = (dev, torch._C._current_graph_task_id())
    pend = _JOBS.get(key)
    if pend is None:
        # [jobs, streams, keep-alive tensors, wgrad calls, device, unit calls, early-reduce stream, queued bytes,
        #  early launches so far]
        pend = _JOBS[key] = [[], [], [], [], dev, [], None, 0.0, 0]
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _flush_jobs(key))
    return pend


def defer_wgrad_call(call: "WgradCall", device: torch.device, *keep: torch.Tensor):
    """Queue a whole weight-gradient call (its operands and workspace kept alive) for this backward's flush."""
    pend = _pending(device)
    pend[3].append(call)
    pend[1].append(torch.cuda.current_stream(pend[4]))
    pend[2].extend(t for t in keep if t is not None)


def flush_deferred_reduces():
    """Run every queued reduce now (callers that drive the kernels outside autograd)."""
    for key in list(_JOBS):
        _flush_jobs(key)


def _p(t: Optional[torch.Tensor]) -> Optional[_VP]:
    return None if t is None else _VP(t.data_ptr())


def dcode(dtype: torch.dtype) -> int:
    if dtype == torch.bfloat16:
        return BF16
    if dtype == torch.float32:
        return F32
    raise ValueError(f"unsupported dtype {dtype} (bf16 / fp32 only)")


_FP16_POLICY = os.environ.get("CAI_FP16_AUTOCAST", "bf16")   # "bf16" | "error"
_FP16_WARNED = False


def set_fp16_autocast_policy(policy: str):
    """What fp16 autocast means for this build: "bf16" (default) computes the region in bf16, "error" raises.

    The reference trains under ``torch.cuda.amp.autocast()`` (fp16, examples/train.py:172,239).  The kernels
    here have bf16 and fp32 paths only (fp32 MFMA accumulation either way); bf16 keeps fp32's exponent range,
    so the fp16 GradScaler the reference pairs with autocast (train.py:174-186) works unchanged -- its scaled
    gradients just never overflow.  A one-time warning says so; "error" restores the strict behaviour."""
    global _FP16_POLICY
    if policy not in ("error", "bf16"):
        raise ValueError(f"fp16 autocast policy must be 'error' or 'bf16', got {policy!r}")
    _FP16_POLICY = policy


def compute_dtype() -> torch.dtype:
    """bf16 inside torch.autocast('cuda', dtype=torch.bfloat16) -- and, by default, inside an fp16 autocast
    region (one warning per process) -- exact fp32 outside autocast."""
    global _FP16_WARNED
    if not torch.is_autocast_enabled("cuda"):
        return torch.float32
    dt = torch.get_autocast_dtype("cuda")
    if dt == torch.bfloat16:
        return dt
    if dt == torch.float16 and _FP16_POLICY == "bf16":
        if not _FP16_WARNED:
            _FP16_WARNED = True
            warnings.warn("compressai (MI355X build): fp16 autocast regions run the bf16 kernels (fp32 accumulate); "
                          "compressai.set_fp16_autocast_policy('error') makes this an error", RuntimeWarning,
                          stacklevel=3)
        return torch.bfloat16
    raise RuntimeError(
        f"autocast dtype {dt} is not supported by the MI355X kernels (bf16 / fp32 only): use "
        "torch.autocast('cuda', dtype=torch.bfloat16), or call "
        "compressai.set_fp16_autocast_policy('bf16') to run fp16 autocast regions in bf16")


def _vec(dtype: torch.dtype) -> int:
    return 8 if dtype == torch.bfloat16 else 4


def _check_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("compressai (MI355X build) runs on GPU tensors only; got a CPU tensor")


def pixel_major_ld(t: torch.Tensor) -> Optional[int]:
    """ld if the 4-D tensor is pixel-major (channel stride 1, pixel stride ld), else None."""
    if t.dim() != 4:
        return None
    B, C, H, W = t.shape
    s = t.stride()
    if C > 1 and s[1] != 1:
        return None
    if W > 1:
        ld = s[3]
    elif H > 1:
        ld = s[2]
    elif B > 1:
        ld = s[0]
    else:
        ld = C
    if ld < C:
        return None
    if (W > 1 and s[3] != ld) or (H > 1 and s[2] != W * ld) or (B > 1 and s[0] != H * W * ld):
        return None
    return int(ld)


def empty_pm(B: int, C: int, H: int, W: int, dtype, device, ld: Optional[int] = None) -> torch.Tensor:
    """Pixel-major [B, C, H, W] tensor (ld = C unless a wider padded row is requested)."""
    ld = C if ld is None else ld
    buf = torch.empty((B, H, W, ld), dtype=dtype, device=device)
    return buf.permute(0, 3, 1, 2)[:, :C]


def to_pm(t: torch.Tensor, dtype: torch.dtype, vec: int) -> Tuple[torch.Tensor, int]:
    """Pixel-major copy/view of a 4-D tensor with ld % vec == 0 (channels zero-padded when C % vec != 0)."""
    B, C, H, W = t.shape
    ld = pixel_major_ld(t)
    if t.dtype == dtype and ld is not None and ld % vec == 0 and (C % vec == 0 or ld > C) and t.data_ptr() % 16 == 0:
        if C % vec == 0 or _pad_is_zero_marked(t):
            return t, ld
    if C % vec == 0:
        out = empty_pm(B, C, H, W, dtype, t.device)
        out.copy_(t)
        return out, C
    cp = (C + 7) // 8 * 8
    src = t.float().contiguous()
    out = empty_pm(B, cp, H, W, dtype, t.device)
    lib.cai_pack_nchw(_p(src), B, C, H, W, dcode(dtype), _p(out), cp, _stream())
    view = out[:, :C]
    _mark_pad_zero(view)
    return view, cp


_ZERO_PAD = "_cai_zero_pad"


def _mark_pad_zero(t):
    setattr(t, _ZERO_PAD, True)


def _pad_is_zero_marked(t):
    return getattr(t, _ZERO_PAD, False)


def as_rows(t: torch.Tensor) -> Tuple[torch.Tensor, int, int, int]:
    """(tensor, ld, npix, C): element (p, c) of the channel-first logical tensor at p*ld + c."""
    C = t.shape[1]
    if t.dim() == 4:
        ld = pixel_major_ld(t)
        if ld is not None:
            npix = t.shape[0] * t.shape[2] * t.shape[3]
            return t, ld, npix, C
    r = t.movedim(1, -1).contiguous()
    return r, C, r.numel() // max(C, 1), C


def empty_rows_like(shape, dtype, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """(logical tensor of `shape` (channel dim 1), its pixel-major buffer)."""
    B, C = shape[0], shape[1]
    buf = torch.empty((B, *shape[2:], C), dtype=dtype, device=device)
    return buf.movedim(-1, 1), buf


# ---------------------------------------------------------------------------
# convolution
# ---------------------------------------------------------------------------

class ConvSpec:
    """Static description of one Conv2d / ConvTranspose2d call site."""

    __slots__ = ("k", "s", "p", "op", "transposed", "act", "act_param", "in_abs", "out_nchw32",
                 "in_mask", "in_mask_param", "act_bwd_downstream")

    def __init__(self, k, s, p, op=0, transposed=False, act=ACT_NONE, act_param=0.0, in_abs=False,
                 out_nchw32=False, in_mask=MASK_NONE, in_mask_param=0.0, act_bwd_downstream=False):
        self.k, self.s, self.p, self.op = int(k), int(s), int(p), int(op)
        self.transposed = bool(transposed)
        self.act, self.act_param = int(act), float(act_param)
        self.in_abs = bool(in_abs)
        self.out_nchw32 = bool(out_nchw32)
        self.in_mask, self.in_mask_param = int(in_mask), float(in_mask_param)
        self.act_bwd_downstream = bool(act_bwd_downstream)


def conv_geom(spec: ConvSpec, B, cin, H, W, cout) -> ConvGeom:
    if spec.transposed:
        OH = (H - 1) * spec.s - 2 * spec.p + spec.k + spec.op
        OW = (W - 1) * spec.s - 2 * spec.p + spec.k + spec.op
    else:
        OH = (H + 2 * spec.p - spec.k) // spec.s + 1
        OW = (W + 2 * spec.p - spec.k) // spec.s + 1
    return ConvGeom(B, cin, H, W, cout, OH, OW, spec.k, spec.s, spec.p, spec.op, int(spec.transposed))


def _pack_weight(g: ConvGeom, dtype, direction: int, weight: torch.Tensor) -> torch.Tensor:
    nbytes = lib.cai_conv_packed_weight_bytes(ctypes.byref(g), dcode(dtype), direction)
    if nbytes == 0:
        raise ValueError("conv: invalid geometry")
    wp = torch.empty(nbytes, dtype=torch.uint8, device=weight.device)
    w = weight.detach().float().contiguous()
    lib.cai_conv_pack_weight(ctypes.byref(g), dcode(dtype), direction, _p(w), None, _p(wp), _stream())
    return wp


def _conv_ws(g: ConvGeom, dtype, direction: int, device):
    nbytes = lib.cai_conv_workspace_bytes(ctypes.byref(g), dcode(dtype), direction)
    if nbytes == 0:
        return None, 0
    return torch.empty(nbytes, dtype=torch.uint8, device=device), nbytes


def _prepack_active():
    from ._prepack import active

    return active()


def _small_deconv(spec: ConvSpec, g: ConvGeom, xld: int, dtype) -> bool:
    """Few-output-channel ConvTranspose2d (x_hat layer): csrc/deconv_small.hip."""
    return (spec.transposed and spec.out_nchw32 and g.out_c <= 16 and spec.act == ACT_NONE and not spec.in_abs
            and spec.in_mask == MASK_NONE and g.in_c % 8 == 0 and xld % 8 == 0
            and lib.cai_deconv_small_workspace_bytes(ctypes.byref(g), dcode(dtype)) > 0)


def _small_ws(g: ConvGeom, dtype, device):
    nbytes = lib.cai_deconv_small_workspace_bytes(ctypes.byref(g), dcode(dtype))
    return torch.empty(nbytes, dtype=torch.uint8, device=device), nbytes


def _small_deconv_bwd(ctx, xpm, weight, gy):
    g, dt = ctx.geom, ctx.dt
    gy = gy.float().contiguous()
    dx = dw = db = None
    if ctx.needs_input_grad[0]:
        ldx = (g.in_c + _vec(dt) - 1) // _vec(dt) * _vec(dt)
        dx = empty_pm(g.batch, g.in_c, g.in_h, g.in_w, dt, gy.device, ld=ldx)
    want_w = ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2])
    wparam, bparam = ctx.params
    direct = want_w and direct_grad(wparam) and (bparam is None or direct_grad(bparam))
    if want_w:
        if direct:
            dw, db = wparam.grad, (bparam.grad if bparam is not None else None)
        else:
            dw = torch.empty(weight.shape, dtype=torch.float32, device=gy.device)
            db = torch.empty(g.out_c, dtype=torch.float32, device=gy.device) if ctx.has_bias else None
    ws, wsb = _small_ws(g, dt, gy.device)
    w32 = weight.detach().float().contiguous()
    fl, nb = _ledger.conv_cost(g, _es(dt), 2, y_bytes=4)
    fl2, nb2 = _ledger.conv_cost(g, _es(dt), 1, y_bytes=4) if dx is not None else (0.0, 0.0)
    _ledger.run(lambda dw=dw, db=db: lib.cai_deconv_small_bwd(ctypes.byref(g), dcode(dt), _p(xpm), ctx.xld, _p(w32),
                                                              _p(gy), _p(dx), ldx if dx is not None else 0, _p(dw),
                                                              _p(db), int(direct), _p(ws), wsb, _stream()),
                "conv_bwd", "deconv_small (im2col + 1x1 GEMMs)", fl + fl2, nb + nb2, dt, _ledger.shape_of(g))
    if direct:
        dw = db = None
    elif dw is not None and weight.dtype != torch.float32:
        dw = dw.to(weight.dtype)
    return dx, dw, db, None


def edge_eligible(k: int, s: int, p: int, cin: int, cout: int, transposed: bool) -> bool:
    """Static part of the edge-layer test (csrc/edge.hip): stride-2 image-side conv / deconv."""
    img_c = cout if transposed else cin
    return s == 2 and k % 2 == 1 and k <= 5 and p == k // 2 and 1 <= img_c <= 3


def _edge_mode(ctx, spec: ConvSpec, g: ConvGeom, dt) -> int:
    """1: analysis first conv (NCHW fp32 image in); 2: synthesis last deconv (NCHW fp32 image out);
    0: the general implicit-GEMM path."""
    if (_EDGE_OFF or dt != torch.bfloat16 or spec.act != ACT_NONE or spec.in_abs or spec.in_mask != MASK_NONE
            or not lib.cai_edge_supported(ctypes.byref(g), dcode(dt))):
        return 0
    if spec.transposed:
        return 2 if spec.out_nchw32 else 0
    return 0 if (spec.out_nchw32 or ctx.needs_input_grad[0]) else 1


def _edge_frag(g: ConvGeom, dt, direction: int, weight: torch.Tensor) -> torch.Tensor:
    """Packed MFMA weight fragments of an edge layer: the model's prepacked copy while its forward is
    active (cai_conv_pack_many), else packed here (one small launch)."""
    packer = _prepack_active()
    frag = packer.lookup(weight, dt, ("edge", direction)) if packer is not None else None
    if frag is None:
        nbytes = lib.cai_edge_frag_bytes(ctypes.byref(g), dcode(dt), direction)
        frag = torch.empty(nbytes, dtype=torch.uint8, device=weight.device)
        lib.cai_edge_pack_weights(ctypes.byref(g), dcode(dt), direction, _p(weight.detach().float().contiguous()),
                                  _p(frag), _stream())
    return frag


def _edge_bwd(ctx, xs, weight, gy):
    g, dt = ctx.geom, ctx.dt
    st = _stream()
    dx = dw = db = None
    if ctx.edge == 1:      # image = x, feature side = dy
        img = xs
        feat, fld = to_pm(gy, dt, 8)
    else:                  # image = dy, feature side = x
        img = gy.float().contiguous()
        feat, fld = xs, ctx.xld
        if ctx.needs_input_grad[0]:
            ldx = (g.in_c + 7) // 8 * 8
            dx = empty_pm(g.batch, g.in_c, g.in_h, g.in_w, dt, gy.device, ld=ldx)
            frag = ctx.frag_bwd if ctx.frag_bwd is not None else _edge_frag(g, dt, 1, weight)
            fl, nb = _ledger.conv_cost(g, _es(dt), 1, y_bytes=4)
            _ledger.run(lambda: lib.cai_edge_deconv_dgrad(ctypes.byref(g), _p(img), _p(frag), _p(dx), ldx, st),
                        "conv_dgrad", "edge_s2d_kernel (deconv dgrad)", fl, nb, dt, _ledger.shape_of(g))
    if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
        wparam, bparam = ctx.params
        direct = direct_grad(wparam) and (bparam is None or direct_grad(bparam))
        if direct:
            dwt, dbt = wparam.grad, (bparam.grad if bparam is not None else None)
        else:
            dwt = torch.empty(weight.shape, dtype=torch.float32, device=gy.device)
            dbt = torch.empty(g.out_c, dtype=torch.float32, device=gy.device) if ctx.has_bias else None
        nbytes = lib.cai_edge_workspace_bytes(ctypes.byref(g), dcode(dt))
        fl, nb = _ledger.conv_cost(g, _es(dt), 2, **({"x_bytes": 4} if ctx.edge == 1 else {"y_bytes": 4}))
        if defer_reduce_ok(direct):
            ws = torch.empty(nbytes, dtype=torch.uint8, device=gy.device)
            job = ReduceJob()
            lib.cai_edge_wgrad_deferred(ctypes.byref(g), _p(img), _p(feat), fld, _p(dwt), _p(dbt), 1, _p(ws),
                                        nbytes, st, ctypes.byref(job))
            defer_job(job, gy.device, ws)
        else:
            with _WgradLaunch(gy.device, direct, img, feat):
                ws = torch.empty(nbytes, dtype=torch.uint8, device=gy.device)
                sw = _stream()
                _ledger.run(lambda: lib.cai_edge_wgrad(ctypes.byref(g), _p(img), _p(feat), fld, _p(dwt), _p(dbt),
                                                       int(direct), _p(ws), nbytes, sw),
                            "conv_wgrad", "edge_wgrad_dma_kernel (+pack, reduce)", fl, nb, dt, _ledger.shape_of(g))
        if not direct:
            dw = dwt if weight.dtype == torch.float32 else dwt.to(weight.dtype)
            db = dbt
    return dx, dw, db, None


def residual_fusable(spec: ConvSpec) -> bool:
    """Whether ConvFn can take a residual input (cai_conv_fwd_res): bf16 pixel-major output of the GEMM kernels,
    activation in this conv's own backward."""
    return (compute_dtype() == torch.bfloat16 and not spec.transposed and not spec.out_nchw32
            and not spec.act_bwd_downstream and not spec.in_abs)


class ConvFn(torch.autograd.Function):
    """y = act(conv(x) + bias [+ res]).  ``res`` (optional, same shape as y) is the residual of ResidualUnit
    (layers.py:211-226: ``out += identity; relu(out)``) added in the conv epilogue before the activation; its
    gradient is the activation-masked output gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, spec: ConvSpec, res=None):
        _check_cuda(x, weight, bias)
        dt = compute_dtype()
        vec = _vec(dt)
        B, cin, H, W = x.shape
        cout = weight.shape[1] if spec.transposed else weight.shape[0]
        g = conv_geom(spec, B, cin, H, W, cout)
        b = bias.detach().float().contiguous() if bias is not None else None
        ctx.spec, ctx.geom, ctx.dt = spec, g, dt
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        ctx.edge = _edge_mode(ctx, spec, g, dt)
        ctx.small = False
        ctx.has_res = res is not None
        ctx.fan = _fan_role(x, "take")
        if res is not None:
            if not residual_fusable(spec) or ctx.edge or tuple(res.shape) != (B, cout, g.out_h, g.out_w):
                raise ValueError(f"conv residual: not fusable for this layer (res {tuple(res.shape)}, "
                                 f"out {(B, cout, g.out_h, g.out_w)}, dtype {dt})")
            _check_cuda(res)
        if ctx.edge == 1:   # space-to-depth first layer: reads the NCHW fp32 image directly
            x32 = x.detach().float().contiguous()
            y = empty_pm(B, cout, g.out_h, g.out_w, dt, x.device)
            frag = _edge_frag(g, dt, 0, weight)
            fl, nb = _ledger.conv_cost(g, _es(dt), 0, x_bytes=4)
            _ledger.run(lambda: lib.cai_edge_conv_fwd(ctypes.byref(g), _p(x32), _p(frag), _p(b), _p(y), cout, _stream()),
                        "conv_fwd", "edge_s2d_kernel (conv fwd)", fl, nb, dt, _ledger.shape_of(g))
            ctx.xld = 0
            ctx.save_for_backward(x32, weight, None)
            return y
        xpm, xld = to_pm(x, dt, vec)
        if ctx.edge == 2:   # depth-to-space last layer: writes the NCHW fp32 image directly
            y = torch.empty((B, cout, g.out_h, g.out_w), dtype=torch.float32, device=x.device)
            frag = _edge_frag(g, dt, 0, weight)
            fl, nb = _ledger.conv_cost(g, _es(dt), 0, y_bytes=4)
            _ledger.run(lambda: lib.cai_edge_deconv_fwd(ctypes.byref(g), _p(xpm), xld, _p(frag), _p(b), _p(y),
                                                        _stream()),
                        "conv_fwd", "edge_d2s_kernel (deconv fwd)", fl, nb, dt, _ledger.shape_of(g))
            packer = _prepack_active()   # the input-gradient fragments of this step's weights
            ctx.frag_bwd = packer.lookup(weight, dt, ("edge", 1)) if packer is not None else None
            ctx.xld = xld
            ctx.save_for_backward(xpm, weight, None)
            return y
        if spec.out_nchw32:
            y = torch.empty((B, cout, g.out_h, g.out_w), dtype=torch.float32, device=x.device)
            ys = (cout * g.out_h * g.out_w, g.out_h * g.out_w, g.out_w, 1)
            ydt = F32
        else:
            y = empty_pm(B, cout, g.out_h, g.out_w, dt, x.device)
            ys = (g.out_h * g.out_w * cout, 1, g.out_w * cout, cout)
            ydt = dcode(dt)
        ctx.small = _small_deconv(spec, g, xld, dt)
        if res is not None:
            rpm, rld = to_pm(res, dt, 4)
            packer = _prepack_active()
            wp = packer.lookup(weight, dt, 0) if packer is not None else None
            ctx.wt_packed = packer.lookup(weight, dt, 1) if packer is not None else None
            if wp is None:
                wp = _pack_weight(g, dt, 0, weight)
            ws, wsb = _conv_ws(g, dt, 0, x.device)
            fl, nb = _ledger.conv_cost(g, _es(dt), 0)
            nb += B * g.out_h * g.out_w * cout * _es(dt)
            _ledger.run(lambda: lib.cai_conv_fwd_res(ctypes.byref(g), dcode(dt), _p(xpm), xld, 0, _p(wp), _p(b),
                                                     spec.act, spec.act_param, _p(rpm), rld, _p(y), ydt, *ys, _p(ws),
                                                     wsb, _stream()),
                        "conv_fwd", _conv_kernel(g, dt, 0, False), fl, nb, dt, _ledger.shape_of(g))
        elif ctx.small:   # few output channels: per-input-pixel GEMM + col2im (csrc/deconv_small.hip)
            ws, wsb = _small_ws(g, dt, x.device)
            w32 = weight.detach().float().contiguous()
            fl, nb = _ledger.conv_cost(g, _es(dt), 0, y_bytes=4)
            _ledger.run(lambda: lib.cai_deconv_small_fwd(ctypes.byref(g), dcode(dt), _p(xpm), xld, _p(w32), _p(b),
                                                         _p(y), _p(ws), wsb, _stream()),
                        "conv_fwd", "deconv_small (GEMM + col2im)", fl, nb, dt, _ledger.shape_of(g))
        else:
            packer = _prepack_active()
            wp = packer.lookup(weight, dt, 0) if packer is not None else None
            ctx.wt_packed = packer.lookup(weight, dt, 1) if packer is not None else None
            if wp is None:
                wp = _pack_weight(g, dt, 0, weight)
            ws, wsb = _conv_ws(g, dt, 0, x.device)
            fl, nb = _ledger.conv_cost(g, _es(dt), 0, y_bytes=4 if spec.out_nchw32 else None)
            _ledger.run(lambda: lib.cai_conv_fwd(ctypes.byref(g), dcode(dt), _p(xpm), xld, int(spec.in_abs), _p(wp),
                                                 _p(b), spec.act, spec.act_param, _p(y), ydt, *ys, _p(ws), wsb,
                                                 _stream()),
                        "conv_fwd", _conv_kernel(g, dt, 0, spec.in_abs), fl, nb, dt, _ledger.shape_of(g))
        ctx.xld = xld
        ctx.save_for_backward(xpm, weight, y if spec.act != ACT_NONE else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        xpm, weight, y = ctx.saved_tensors
        spec, g, dt = ctx.spec, ctx.geom, ctx.dt
        vec = _vec(dt)
        code = dcode(dt)
        st = _stream()
        if ctx.edge:
            return _edge_bwd(ctx, xpm, weight, gy) + (None,)
        if ctx.small:
            return _small_deconv_bwd(ctx, xpm, weight, gy) + (None,)
        gpm, gld = to_pm(gy, dt, vec)
        if spec.act != ACT_NONE and not spec.act_bwd_downstream and not getattr(ctx, "gy_masked", False):
            mode = 1 if spec.act == 1 else 2
            out = empty_pm(g.batch, g.out_c, g.out_h, g.out_w, dt, gy.device)
            yld = pixel_major_ld(y)
            n_el = g.batch * g.out_h * g.out_w * g.out_c
            _ledger.run(lambda gpm=gpm, gld=gld: lib.cai_act_bwd(mode, spec.act_param, _p(y), yld, _p(gpm), gld,
                                                                 _p(out), g.out_c, g.batch * g.out_h * g.out_w,
                                                                 g.out_c, code, st),
                        "act_bwd", "act_bwd_kernel", 0, 3 * n_el * _es(dt), dt)
            gpm, gld = out, g.out_c
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wt = ctx.wt_packed if getattr(ctx, "wt_packed", None) is not None else _pack_weight(g, dt, 1, weight)
            ldx = (g.in_c + vec - 1) // vec * vec
            dx = empty_pm(g.batch, g.in_c, g.in_h, g.in_w, dt, gy.device, ld=ldx)
            aux = xpm if spec.in_mask != MASK_NONE else None
            ws, wsb = _conv_ws(g, dt, 1, gy.device)
            fl, nb = _ledger.conv_cost(g, _es(dt), 1)
            # ResidualChainFn: + the residual's gradient in the epilogue (then the previous unit's ReLU mask)
            dres = getattr(ctx, "dx_res", None)
            rmask = getattr(ctx, "dx_res_mask", MASK_NONE)
            dres2 = getattr(ctx, "dx_res2", None)   # AttentionBlockFn: + the other branch's / the gate's gradient
            if dres is None and dres2 is not None:
                dres, dres2 = dres2, None
            fan, done = getattr(ctx, "fan", None), False
            if fan is not None and fan.pending is not None and dres is None and dt == torch.bfloat16 and ldx % 8 == 0:
                # FanOutFn: the input's other consumer has run its backward -- its gradient joins this dgrad's
                # epilogue (after the input mask: dx = mask(x) * conv_input_grad + other) instead of a separate add
                post = fan.pending
                if aux is None:
                    dres, fan.pending = post, None
                elif "halo" not in _conv_kernel(g, dt, 1)():
                    ppm, pld = to_pm(post, dt, 4)
                    mode = spec.in_mask | MASK_BEFORE_RES
                    _ledger.run(lambda ppm=ppm, dx=dx, wt=wt, gpm=gpm, ws=ws: lib.cai_conv_dgrad_res(
                                    ctypes.byref(g), code, _p(gpm), gld, _p(wt), _p(ppm), pld, _p(dx), ldx, mode,
                                    spec.in_mask_param, _p(xpm), ctx.xld, _p(ws), wsb, st),
                                "conv_dgrad", _conv_kernel(g, dt, 1), fl, nb + post.numel() * _es(dt), dt,
                                _ledger.shape_of(g))
                    fan.pending, done = None, True
            if done:
                pass
            elif dres is not None and dt == torch.bfloat16 and aux is None and ldx % 8 == 0:
                rpm, rld = to_pm(dres, dt, 4)
                maux = xpm if rmask != MASK_NONE else None
                if dres2 is not None:
                    r2pm, r2ld = to_pm(dres2, dt, 4)
                    _ledger.run(lambda: lib.cai_conv_dgrad_res2(ctypes.byref(g), code, _p(gpm), gld, _p(wt), _p(rpm),
                                                                rld, _p(r2pm), r2ld, _p(dx), ldx, rmask, 0.0,
                                                                _p(maux), ctx.xld if maux is not None else 0, _p(ws),
                                                                wsb, st),
                                "conv_dgrad", _conv_kernel(g, dt, 1), fl, nb, dt, _ledger.shape_of(g))
                else:
                    _ledger.run(lambda: lib.cai_conv_dgrad_res(ctypes.byref(g), code, _p(gpm), gld, _p(wt), _p(rpm),
                                                               rld, _p(dx), ldx, rmask, 0.0, _p(maux),
                                                               ctx.xld if maux is not None else 0, _p(ws), wsb, st),
                                "conv_dgrad", _conv_kernel(g, dt, 1), fl, nb, dt, _ledger.shape_of(g))
            else:
                _ledger.run(lambda: lib.cai_conv_dgrad(ctypes.byref(g), code, _p(gpm), gld, _p(wt), _p(dx), ldx,
                                                       spec.in_mask, spec.in_mask_param, _p(aux),
                                                       ctx.xld if aux is not None else 0, _p(ws), wsb, st),
                            "conv_dgrad", _conv_kernel(g, dt, 1), fl, nb, dt, _ledger.shape_of(g))
                if dres is not None:
                    dx = dx + dres
                if dres2 is not None:
                    dx = dx + dres2
                if rmask != MASK_NONE:
                    raise RuntimeError("conv dgrad: a residual-gradient mask needs the fused bf16 path")
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            wparam, bparam = ctx.params
            dw, db = conv_wgrad(g, dt, xpm, ctx.xld, int(spec.in_abs), gpm, gld, wparam, bparam, weight,
                                ctx.has_bias)
        dres = None
        if ctx.has_res and ctx.needs_input_grad[4]:
            dres = gpm
        return dx, dw, db, None, dres


_BATCHED_WGRAD = {}
# the weight-gradient kernels whose calls are deferred to the backward's flush and batched there (one launch per
# kernel variant, cai_conv_wgrad_batch): the latent-size kernel and the pixel-split kernels of the mid-size and
# stride-1 3x3 layers (cheng2020: 12 + 15 launches per step).  The stride-2 halo weight gradients of the big maps
# stay in place: each already fills the chip, and right after its input gradient its operands are cache-warm.
_BATCHED_WGRAD_KERNELS = (b"wgrad_small_kernel", b"wgrad_glds_kernel<256>", b"wgrad_glds_kernel<128>",
                          b"wgrad_halo_kernel<3,s1>")


def _small_wgrad(g, code, in_abs) -> bool:
    """Whether this weight gradient's call is deferred and batched (_BATCHED_WGRAD_KERNELS)."""
    key = (tuple(getattr(g, f) for f, _ in ConvGeom._fields_), code, int(in_abs))
    v = _BATCHED_WGRAD.get(key)
    if v is None:
        name = lib.cai_conv_kernel_name(ctypes.byref(g), code, 2, int(in_abs))
        v = _BATCHED_WGRAD[key] = name in _BATCHED_WGRAD_KERNELS
    return v


def conv_wgrad(g, dt, xpm, xld, in_abs, gpm, gld, wparam, bparam, weight, has_bias):
    """Weight (+ bias) gradient of one conv from its input xpm and output gradient gpm (pixel-major): straight
    into the optimizer's flat buffer when the parameters are direct_grad (returns None, None; the final reduce
    deferred to the end of the backward), else fresh tensors."""
    code = dcode(dt)
    dev = gpm.device
    nbytes = lib.cai_conv_wgrad_workspace_bytes(ctypes.byref(g), code)
    # a weight passed as a same-size view of its parameter (Linear's [out, in] weight viewed [out, in, 1, 1]): its
    # gradient lands in the parameter's flat-buffer slot through the same view (autograd's add into .grad skipped)
    wbase = getattr(wparam, "_base", None)
    wdir = wparam if direct_grad(wparam) else (
        wbase if wbase is not None and wbase.numel() == wparam.numel() and direct_grad(wbase) else None)
    direct = wdir is not None and (bparam is None or direct_grad(bparam))
    if direct:   # accumulate straight into the optimizer's flat gradient buffer
        dw = wdir.grad if wdir is wparam else wdir.grad.view(wparam.shape)
        db = bparam.grad if bparam is not None else None
    else:
        dw = torch.empty(weight.shape, dtype=torch.float32, device=dev)
        db = torch.empty(g.out_c, dtype=torch.float32, device=dev) if has_bias else None
    fl, nb = _ledger.conv_cost(g, _es(dt), 2)
    st = _stream()
    if defer_reduce_ok(direct) and _WGRAD_BATCH and not _WGRAD_SIDE_PX and _small_wgrad(g, code, in_abs):
        wws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        call = WgradCall(g, code, _p(xpm), xld, int(in_abs), 0, _p(gpm), gld, _p(dw), _p(db), 1, _p(wws), nbytes)
        defer_wgrad_call(call, dev, xpm, gpm, wws)
    elif defer_reduce_ok(direct):
        npix = g.batch * (g.in_h * g.in_w if g.transposed else g.out_h * g.out_w)
        with _SideDeferred(dev, npix, xpm, gpm):
            wws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            job = ReduceJob()
            lib.cai_conv_wgrad_deferred(ctypes.byref(g), code, _p(xpm), xld, int(in_abs), 0, _p(gpm), gld, _p(dw),
                                        _p(db), 1, _p(wws), nbytes, _stream(), ctypes.byref(job))
            defer_job(job, dev, wws)
    else:
        with _WgradLaunch(dev, direct, xpm, gpm):
            wws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            sw = _stream()
            _ledger.run(lambda: lib.cai_conv_wgrad(ctypes.byref(g), code, _p(xpm), xld, int(in_abs), 0, _p(gpm), gld,
                                                   _p(dw), _p(db), int(direct), _p(wws), nbytes, sw),
                        "conv_wgrad", _conv_kernel(g, dt, 2, in_abs), fl, nb, dt, _ledger.shape_of(g))
    if direct:
        return None, None
    if weight.dtype != torch.float32:
        dw = dw.to(weight.dtype)
    return dw, db


class _SubCtx:
    """A stand-in autograd ctx: lets a multi-conv autograd node run ConvFn's forward / backward per layer."""

    def __init__(self, needs):
        self.needs_input_grad = needs
        self.saved_tensors = ()

    def save_for_backward(self, *tensors):
        self.saved_tensors = tensors


class _FanIn:
    """The gradient hand-off of FanOutFn: the giving consumer's backward leaves its input gradient here; the taking
    consumer's backward, when it runs later, adds it in its own dgrad epilogue; FanOutFn adds what is left."""

    __slots__ = ("pending",)

    def __init__(self):
        self.pending = None


_FAN_ATTR = "_cai_fan"


def _fan_role(x, role):
    f = getattr(x, _FAN_ATTR, None)
    return f[0] if f is not None and f[1] == role else None


class FanOutFn(torch.autograd.Function):
    """x -> (x_take, x_give): two aliases of one tensor read by two consumers (the hyperprior models' y: h_a's
    first conv and the GaussianConditional), so that their gradients meet in a kernel rather than in autograd's
    input buffer (an ATen add per step).  The GaussianConditional (giver) hands its x gradient over instead of
    returning it; the conv (taker), whose backward runs after it (h_a's gradient arrives through the scales),
    adds it in its dgrad epilogue (cai_conv_dgrad_res: CAI_MASK_BEFORE_RES under h_a's abs mask).  Whatever is
    not absorbed -- another order, a layout the epilogue cannot take -- is added here.  Values are autograd's:
    dx = dx_take + dx_give."""

    @staticmethod
    def forward(ctx, x, box, n: int):
        ctx.set_materialize_grads(False)
        ctx.box = box
        return tuple(x.view_as(x) for _ in range(n))

    @staticmethod
    def backward(ctx, *grads):
        box = ctx.box
        extra, box.pending = box.pending, None
        gs = [t for t in (*grads, extra) if t is not None]
        if not gs:
            return None, None, None
        total = gs[0]
        for t in gs[1:]:
            total = _add_grads(total, t)
        return total, None, None


def _add_grads(a, b):
    """a + b for two gradients of one tensor: the native add for bf16 pixel-major, else torch."""
    if a.dtype == b.dtype == torch.bfloat16 and a.is_cuda and a.dim() == 4 and a.shape == b.shape:
        ap, ald = to_pm(a, torch.bfloat16, 4)
        bp, bld = to_pm(b, torch.bfloat16, 4)
        y, yld = _out_pm_like(a, torch.bfloat16)
        B, C, H, W = a.shape
        _ledger.run(lambda ap=ap, bp=bp, y=y: lib.cai_add_act(BF16, _p(ap), ald, _p(bp), bld, _p(y), yld, B * H * W,
                                                             C, ACT_NONE, 0.0, _stream()),
                    "add_act", "add_act_kernel", 0, 3 * B * H * W * C * 2, torch.bfloat16)
        return y
    return a + b


_FANOUT = os.environ.get("CAI_FANOUT", "1") == "1"   # 0: autograd sums the gradients (A/B)


def fan_out(x, n: int = 2, absorb: bool = True):
    """n aliases of x for its n consumers (x itself n times when x does not require a gradient); their gradients
    are summed by the native add instead of autograd's ATen add.  absorb (n == 2): the first alias is read by a
    conv (taker), the second by a GaussianConditional (giver), whose gradient the conv adds in its dgrad epilogue.
    absorb=False keeps the sum order-independent (one native add of the two gradients, whichever stream or order
    produced them: bit-identical to autograd's sum)."""
    if not (_FANOUT and torch.is_grad_enabled() and x.requires_grad):
        return (x,) * n
    box = _FanIn()
    outs = FanOutFn.apply(x, box, n)
    if absorb and n == 2:
        setattr(outs[0], _FAN_ATTR, (box, "take"))
        setattr(outs[1], _FAN_ATTR, (box, "give"))
    return outs


class ResidualChainFn(torch.autograd.Function):
    """A chain of ResidualUnits (layers.py:211-226; AttentionBlock's conv_a / conv_b, :225-236) as one autograd
    node.  Unit k: y_k = relu(conv1x1(relu(conv3x3(relu(conv1x1(y_{k-1}))))) + y_{k-1}), every ReLU in a conv
    epilogue (the residual add in the last conv's, cai_conv_fwd_res), every ReLU mask in the next conv's dgrad
    epilogue.  Backward: a unit input's two gradients (through the convs and through the residual) are summed in
    the first conv's dgrad epilogue (cai_conv_dgrad_res), which inside the chain also applies the previous unit's
    trailing ReLU mask (y_{k-1} > 0) -- so only the chain's last unit runs an activation-backward launch.  Same
    kernels and arithmetic as the per-layer ConvFn chain otherwise.

    params: (w0, b0, w2, b2, w4, b4) per unit; specs: ((s0, s2, s4), ...) per unit; out_masked: the chain's
    consumer applies the last unit's ReLU mask to the gradient it returns."""

    @staticmethod
    def forward(ctx, x, specs, out_masked, *params):
        need = ctx.needs_input_grad   # (x, specs, out_masked, *params)
        y, ctx.subs = _chain_forward(x, specs, out_masked, params, need[0], need[3:])
        _stash(ctx, _unit_ctxs(ctx.subs))
        return y

    @staticmethod
    def backward(ctx, gy):
        with _unstash(ctx):
            g, flat = _chain_backward(ctx.subs, gy)
        return (g, None, None, *flat)


def _stash(ctx, subs):
    """Every stand-in context's tensors through ctx.save_for_backward (version-counter checks, no y -> grad_fn ->
    ctx -> y reference cycle); the stand-ins keep only metadata between forward and backward."""
    flat, counts = [], []
    for c in subs:
        counts.append(len(c.saved_tensors))
        flat.extend(c.saved_tensors)
        c.saved_tensors = ()
    ctx.save_for_backward(*flat)
    ctx.stash = (subs, counts)


class _unstash:
    """Hand the stand-in contexts their saved tensors for one backward (retain_graph: a second backward restores
    them from ctx.saved_tensors again)."""

    def __init__(self, ctx):
        self.subs, counts = ctx.stash
        saved, i = ctx.saved_tensors, 0
        for c, n in zip(self.subs, counts):
            c.saved_tensors = tuple(saved[i:i + n])
            i += n

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        for c in self.subs:
            c.saved_tensors = ()
            c.dx_res = c.dx_res2 = None
        return False


# One launch per ResidualUnit and direction (csrc/resunit.hip) instead of three conv launches: bf16, N in {128, 192}.
# CAI_RESUNIT_FUSED=0 keeps the per-conv chain (A/B).
_RESUNIT_FUSED = os.environ.get("CAI_RESUNIT_FUSED", "1") == "1"
_RESUNIT_WGRAD = os.environ.get("CAI_RESUNIT_WGRAD", "1") == "1"   # one launch for the unit's weight gradients
_SPEC_1x1, _SPEC_3x3 = ConvSpec(1, 1, 0), ConvSpec(3, 1, 1)


class _FusedUnit:
    """A ResidualUnit run by cai_resunit: saved tensors (x, h1, h2, y) and what its backward needs."""

    __slots__ = ("saved_tensors", "params", "geoms", "gy_masked", "mask_x", "dx_res2", "dx_res", "need_x", "wt_packed")

    def __init__(self, params, geoms, need_x):
        self.params, self.geoms, self.need_x = params, geoms, need_x
        self.saved_tensors = ()
        self.wt_packed = None
        self.gy_masked = self.mask_x = False
        self.dx_res2 = self.dx_res = None


def _gdn_name(code, npix, C, ld, direction) -> str:
    """The GDN kernel a call launches (ledger label); "gdn" from an older library without the query (A/B)."""
    try:
        return lib.cai_gdn_kernel_name(code, npix, C, ld, C, direction).decode()
    except AttributeError:
        return "gdn_fwd" if direction == 0 else "gdn_bwd"


_HAS = {}


def _has_resunit() -> bool:
    """The library has the fused unit kernels (an older one in an A/B run does not: per-conv chain)."""
    v = _HAS.get("resunit")
    if v is None:
        v = _HAS["resunit"] = hasattr(lib.load(), "cai_resunit")
    return v


def _resunit_ok(y, specs, params) -> bool:
    if not _RESUNIT_FUSED or compute_dtype() != torch.bfloat16 or y.dim() != 4 or not y.is_cuda or not _has_resunit():
        return False
    n = y.shape[1]
    w0, b0, w2, b2, w4, b4 = params
    return (n in (128, 192) and b0 is not None and b2 is not None and b4 is not None
            and tuple(w0.shape) == (n // 2, n, 1, 1) and tuple(w2.shape) == (n // 2, n // 2, 3, 3)
            and tuple(w4.shape) == (n, n // 2, 1, 1)
            and (specs[1].k, specs[1].s, specs[1].p) == (3, 1, 1))


def _packed_kp(weight, g, dt, direction):
    """The layer's packed MFMA operand for `direction` (the model's prepacked copy when its forward is active) and
    its row length."""
    packer = _prepack_active()
    wp = packer.lookup(weight, dt, direction) if packer is not None else None
    if wp is None:
        wp = _pack_weight(g, dt, direction, weight)
    kout = g.out_c if direction == 0 else g.in_c
    return wp, wp.numel() // (2 * ((kout + 15) // 16 * 16))


def _resunit_fwd(y, params, need_x):
    dt = torch.bfloat16
    xpm, xld = to_pm(y, dt, 8)
    B, n, H, W = xpm.shape
    nh = n // 2
    w0, b0, w2, b2, w4, b4 = params
    ga = conv_geom(_SPEC_1x1, B, n, H, W, nh)
    gb = conv_geom(_SPEC_3x3, B, nh, H, W, nh)
    gc = conv_geom(_SPEC_1x1, B, nh, H, W, n)
    (wa, kpa), (wb, kpb), (wc, kpc) = (_packed_kp(w0, ga, dt, 0), _packed_kp(w2, gb, dt, 0),
                                       _packed_kp(w4, gc, dt, 0))
    h1 = empty_pm(B, nh, H, W, dt, xpm.device)
    h2 = empty_pm(B, nh, H, W, dt, xpm.device)
    out = empty_pm(B, n, H, W, dt, xpm.device)
    bs = [b.detach().float().contiguous() for b in (b0, b2, b4)]
    A = ResunitArgs(batch=B, h=H, w=W, n=n, x=xpm.data_ptr(), wa=wa.data_ptr(), wb=wb.data_ptr(), wc=wc.data_ptr(),
                    ba=bs[0].data_ptr(), bb=bs[1].data_ptr(), bc=bs[2].data_ptr(), h1=h1.data_ptr(),
                    h2=h2.data_ptr(), out=out.data_ptr(), x_ld=xld, out_ld=n, kpa=kpa, kpb=kpb, kpc=kpc)
    fl = sum(_ledger.conv_cost(g, 2, 0)[0] for g in (ga, gb, gc))
    # the closure owns every buffer A points at: the ledger may replay it after the step (bench.py --replay)
    _ledger.run(lambda keep=(A, xpm, wa, wb, wc, h1, h2, out, bs): lib.cai_resunit(ctypes.byref(keep[0]), 0, _stream()),
                "conv_fwd", f"resunit_kernel<{n},fwd>", fl, 2 * B * H * W * (2 * n + 2 * nh), dt,
                f"ResidualUnit N={n} {H}x{W} B={B}")
    u = _FusedUnit(params, (ga, gb, gc), need_x)
    u.saved_tensors = (xpm, h1, h2, out)
    if _prepack_active() is not None:
        # the input-gradient operands from this forward's pack_many launch: the backward runs after the forward's
        # prepack context has closed, where a lookup would miss and pack each of them in a launch of its own
        u.wt_packed = (_packed_kp(w4, gc, dt, 1), _packed_kp(w2, gb, dt, 1), _packed_kp(w0, ga, dt, 1))
    return out, u


def _resunit_bwd(u: "_FusedUnit", gy):
    dt = torch.bfloat16
    xpm, h1, h2, y = u.saved_tensors
    ga, gb, gc = u.geoms
    w0, b0, w2, b2, w4, b4 = u.params
    B, n, H, W = xpm.shape
    nh = n // 2
    gpm, gld = to_pm(gy, dt, 8)
    wt = getattr(u, "wt_packed", None)
    (wa, kpa), (wb, kpb), (wc, kpc) = wt if wt is not None else (_packed_kp(w4, gc, dt, 1), _packed_kp(w2, gb, dt, 1),
                                                                 _packed_kp(w0, ga, dt, 1))
    dev = xpm.device
    g_c = None if u.gy_masked else empty_pm(B, n, H, W, dt, dev)
    g_b = empty_pm(B, nh, H, W, dt, dev)
    g_a = empty_pm(B, nh, H, W, dt, dev)
    dx = empty_pm(B, n, H, W, dt, dev)
    res2 = None
    if u.dx_res2 is not None:
        res2, r2ld = to_pm(u.dx_res2, dt, 4)
    yld = pixel_major_ld(y)
    A = ResunitArgs(batch=B, h=H, w=W, n=n, x=gpm.data_ptr(), y=y.data_ptr(), wa=wa.data_ptr(), wb=wb.data_ptr(),
                    wc=wc.data_ptr(), h1=h1.data_ptr(), h2=h2.data_ptr(), out=dx.data_ptr(),
                    gc=g_c.data_ptr() if g_c is not None else None, gb=g_b.data_ptr(), ga=g_a.data_ptr(),
                    res2=res2.data_ptr() if res2 is not None else None,
                    xmask=xpm.data_ptr() if u.mask_x else None, x_ld=gld, y_ld=yld, out_ld=n,
                    res2_ld=r2ld if res2 is not None else 0, xmask_ld=pixel_major_ld(xpm) if u.mask_x else 0,
                    kpa=kpa, kpb=kpb, kpc=kpc, gy_masked=int(u.gy_masked))
    fl = sum(_ledger.conv_cost(g, 2, 1)[0] for g in (ga, gb, gc))
    _ledger.run(lambda keep=(A, gpm, y, wa, wb, wc, h1, h2, dx, g_c, g_b, g_a, res2, xpm):
                lib.cai_resunit(ctypes.byref(keep[0]), 1, _stream()), "conv_dgrad", f"resunit_kernel<{n},bwd>", fl,
                2 * B * H * W * (3 * n + 4 * nh), dt, f"ResidualUnit N={n} {H}x{W} B={B}")
    gcc, gcld = (gpm, gld) if g_c is None else (g_c, n)
    if _RESUNIT_WGRAD and hasattr(lib.load(), "cai_resunit_wgrad"):
        grads = _resunit_wgrad(u, xpm, h1, h2, g_a, g_b, gcc, gcld)
        return dx, grads
    dw4, db4 = conv_wgrad(gc, dt, h2, nh, 0, gcc, gcld, w4, b4, w4, True)
    dw2, db2 = conv_wgrad(gb, dt, h1, nh, 0, g_b, nh, w2, b2, w2, True)
    dw0, db0 = conv_wgrad(ga, dt, xpm, pixel_major_ld(xpm), 0, g_a, nh, w0, b0, w0, True)
    return dx, (dw0, db0, dw2, db2, dw4, db4)


def _resunit_wgrad(u: "_FusedUnit", xpm, h1, h2, g_a, g_b, gcc, gcld):
    """The unit's six parameter gradients in one launch (cai_resunit_wgrad, csrc/resunit.hip) + three WGRAD
    reduce jobs: deferred to the end of the backward when every parameter writes straight into the optimizer's
    flat buffer (as conv_wgrad), else run now into fresh tensors."""
    w0, b0, w2, b2, w4, b4 = u.params
    B, n, H, W = xpm.shape
    dev = xpm.device
    direct = all(direct_grad(p) for p in u.params)
    if direct:
        outs = [p.grad for p in u.params]
    else:
        outs = [torch.empty(p.shape, dtype=torch.float32, device=dev) for p in u.params]
    dw0, db0, dw2, db2, dw4, db4 = outs
    A = ResunitWgradArgs(batch=B, h=H, w=W, n=n, x=xpm.data_ptr(), h1=h1.data_ptr(), h2=h2.data_ptr(),
                         ga=g_a.data_ptr(), gb=g_b.data_ptr(), gc=gcc.data_ptr(), x_ld=pixel_major_ld(xpm),
                         gc_ld=gcld, dwa=dw0.data_ptr(), dba=db0.data_ptr(), dwb=dw2.data_ptr(), dbb=db2.data_ptr(),
                         dwc=dw4.data_ptr(), dbc=db4.data_ptr(), accumulate=int(direct))
    nbytes = lib.cai_resunit_wgrad_workspace_bytes(ctypes.byref(A))
    st = _stream()
    if defer_reduce_ok(direct) and _WGRAD_BATCH and not _WGRAD_SIDE_PX:
        wws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        pend = _pending(dev)
        pend[5].append((A, wws.data_ptr(), nbytes))
        pend[1].append(torch.cuda.current_stream(pend[4]))
        pend[2].extend((xpm, h1, h2, g_a, g_b, gcc, wws))
    elif defer_reduce_ok(direct):
        with _SideDeferred(dev, B * H * W, xpm, h1, h2, g_a, g_b, gcc):
            wws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            jobs = (ReduceJob * 3)()
            lib.cai_resunit_wgrad(ctypes.byref(A), _p(wws), nbytes, _stream(), jobs)
            for j in jobs:
                defer_job(j, dev, wws)
    else:
        wws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        nh = n // 2
        P = B * H * W
        fl = 2.0 * P * (nh * n * 2 + 9 * nh * nh)
        nb = 2 * P * (3 * n + 4 * nh)
        _ledger.run(lambda keep=(A, wws, xpm, h1, h2, g_a, g_b, gcc, outs):
                    lib.cai_resunit_wgrad(ctypes.byref(keep[0]), _p(keep[1]), nbytes, st, None), "conv_wgrad",
                    f"resunit_wgrad_kernel<{n}> (+reduce)", fl, nb, torch.bfloat16,
                    f"ResidualUnit N={n} {H}x{W} B={B}")
    if direct:
        return (None,) * 6
    return tuple(o if p.dtype == torch.float32 else o.to(p.dtype) for o, p in zip(outs, u.params))


def _chain_forward(x, specs, out_masked, params, x_need, p_need):
    subs = []
    y = x
    for k, (s0, s2, s4) in enumerate(specs):
        pr = params[6 * k:6 * k + 6]
        if _resunit_ok(y, (s0, s2, s4), pr):
            y, u = _resunit_fwd(y, pr, x_need or k > 0)
            if k > 0:   # this unit's input is the previous unit's ReLU output: mask its gradient here
                u.mask_x = True
                prev = subs[-1]
                if isinstance(prev, _FusedUnit):
                    prev.gy_masked = True
                else:
                    prev[2].gy_masked = True
            subs.append(u)
            continue
        w0, b0, w2, b2, w4, b4 = pr
        pn = p_need[6 * k:6 * k + 6]
        c0 = _SubCtx((x_need or k > 0, pn[0], pn[1], False, False))
        c2 = _SubCtx((True, pn[2], pn[3], False, False))
        c4 = _SubCtx((True, pn[4], pn[5], False, True))
        h = ConvFn.forward(c0, y, w0, b0, s0)
        h = ConvFn.forward(c2, h, w2, b2, s2)
        y = ConvFn.forward(c4, h, w4, b4, s4, y)
        if k > 0:   # this unit's input is the previous unit's ReLU output: mask its gradient here
            prev = subs[-1]
            if isinstance(prev, _FusedUnit):
                # a fused unit hands its gradient over unmasked only through dx; the mask goes here
                c0.dx_res_mask = MASK_POS
                prev.gy_masked = True
            else:
                c0.dx_res_mask = MASK_POS
                prev[2].gy_masked = True
        subs.append((c0, c2, c4))
    if out_masked:   # the consumer (a MASK_POS dgrad, GateFn relu_a) hands back the masked gradient
        last = subs[-1]
        if isinstance(last, _FusedUnit):
            last.gy_masked = True
        else:
            last[2].gy_masked = True
    return y, subs


def _unit_ctxs(subs):
    """Every stand-in context of a chain (a fused unit is one)."""
    out = []
    for u in subs:
        out.extend([u] if isinstance(u, _FusedUnit) else list(u))
    return out


def _chain_backward(subs, gy, dx_res2=None, before_first=None):
    """-> (gradient of the chain input, flat parameter gradients); dx_res2: one more gradient of the chain input,
    summed in the first unit's dgrad epilogue (a callable: evaluated right before that unit, after
    `before_first()`, so another stream's producer can run under the later units)."""
    grads = []
    g = gy
    for k in range(len(subs) - 1, -1, -1):
        if k == 0 and before_first is not None:
            before_first()
        if k == 0 and callable(dx_res2):
            dx_res2 = dx_res2()
        u = subs[k]
        if isinstance(u, _FusedUnit):
            if k == 0 and dx_res2 is not None:
                u.dx_res2 = dx_res2
            g, pg = _resunit_bwd(u, g)
            grads.append(pg)
            continue
        c0, c2, c4 = u
        dh2, dw4, db4, _, g4 = ConvFn.backward(c4, g)
        dh1, dw2, db2, _, _ = ConvFn.backward(c2, dh2)
        c0.dx_res = g4
        if k == 0 and dx_res2 is not None:
            c0.dx_res2 = dx_res2
        g, dw0, db0, _, _ = ConvFn.backward(c0, dh1)
        grads.append((dw0, db0, dw2, db2, dw4, db4))
    return g, [t for unit in reversed(grads) for t in unit]


class ResidualBlockFn(torch.autograd.Function):
    """ResidualBlock with an identity skip (layers.py:162-193): y = leaky(conv2(leaky(conv1(x)))) + x as one
    autograd node.  x's two gradients (through the convs and through the skip) are summed in conv1's dgrad
    epilogue (cai_conv_dgrad_res) instead of an autograd gradient-sum launch; the forward runs the same kernels as
    the per-module chain (conv1 with its LeakyReLU epilogue, conv2 applying that mask in its dgrad, the add)."""

    @staticmethod
    def forward(ctx, x, spec1, spec2, w1, b1, w2, b2):
        need = ctx.needs_input_grad   # (x, spec1, spec2, w1, b1, w2, b2)
        c1 = _SubCtx((need[0], need[3], need[4], False, False))
        c2 = _SubCtx((True, need[5], need[6], False, False))
        h = ConvFn.forward(c1, x, w1, b1, spec1)
        o = ConvFn.forward(c2, h, w2, b2, spec2)
        y = AddActFn.forward(_SubCtx((True, True, False, False)), o, x, ACT_NONE, 0.0)
        ctx.c1, ctx.c2 = c1, c2
        _stash(ctx, [c1, c2])
        return y

    @staticmethod
    def backward(ctx, gy):
        with _unstash(ctx):
            dh, dw2, db2, _, _ = ConvFn.backward(ctx.c2, gy)
            ctx.c1.dx_res = gy   # the skip's gradient (the add has no activation)
            dx, dw1, db1, _, _ = ConvFn.backward(ctx.c1, dh)
        return dx, None, None, dw1, db1, dw2, db2


# AttentionBlock branches (and the skip branches of ResidualBlockWithStride / ResidualBlockUpsample) on two streams
# when their launches are small (<= CAI_AB_STREAM_PX input pixels: C4's 16 x 16 latents at B = 4 run the units on 16
# blocks, its 64 x 64 maps on 256; profiles/r04_attention_two_streams_ab.log); CAI_AB_STREAM=0 keeps them serial
_AB_STREAM = os.environ.get("CAI_AB_STREAM", "1") == "1"
_AB_STREAM_PX = int(os.environ.get("CAI_AB_STREAM_PX", "16384"))
_AB_SIDE = {}


def _ab_side(x, params=()):
    """The side stream for a small branch, or None.  `params`: the parameters of a branch that is its own autograd
    node (a module called on the side stream): its gradients must go straight into FusedAdam's buffer (direct
    grads) -- a gradient returned to an AccumulateGrad node of the caller's stream would cross streams (torch
    syncs it, warns, and such a step could not be graph-captured)."""
    if not (_AB_STREAM and x.is_cuda and _ledger.active() is None):
        return None
    B, _, H, W = x.shape
    if B * H * W > _AB_STREAM_PX:
        return None
    if torch.is_grad_enabled() and any(p.requires_grad and not direct_grad(p) for p in params):
        return None
    s = _AB_SIDE.get(x.device)
    if s is None:
        s = _AB_SIDE[x.device] = torch.cuda.Stream(device=x.device)
    return s


class AttentionBlockFn(torch.autograd.Function):
    """AttentionBlock (layers.py:196-244) as one autograd node: y = a * sigmoid(b) + x with a = conv_a(x) and
    b = conv_b(x) (three ResidualUnits each, as in ResidualChainFn; conv_b's 1x1 conv after its chain).  x's three
    gradients (both branches and the gate's identity) are summed in the first conv dgrad epilogues (conv_b's first
    unit: + the gate's; conv_a's first unit: + conv_b's) -- no gradient-sum launch.

    params: conv_a's 18, conv_b's 18 (6 per unit as in ResidualChainFn), then conv_b[3]'s weight and bias."""

    @staticmethod
    def forward(ctx, x, specs_a, specs_b, spec_b3, *params):
        need = ctx.needs_input_grad   # (x, specs_a, specs_b, spec_b3, *params)
        pa, pb, (w3, b3) = params[:18], params[18:36], params[36:38]
        c3 = _SubCtx((True, need[40], need[41], False, False))
        side = _ab_side(x)
        ctx.side = side
        if side is None:
            a, ctx.sub_a = _chain_forward(x, specs_a, True, pa, need[0], need[4:22])
            hb, ctx.sub_b = _chain_forward(x, specs_b, True, pb, need[0], need[22:40])
            bb = ConvFn.forward(c3, hb, w3, b3, spec_b3)
        else:
            # small maps: the two branches' launches fill a fraction of the GPU each -- branch b on the side stream
            main = torch.cuda.current_stream(x.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                hb, ctx.sub_b = _chain_forward(x, specs_b, True, pb, need[0], need[22:40])
                bb = ConvFn.forward(c3, hb, w3, b3, spec_b3)
            a, ctx.sub_a = _chain_forward(x, specs_a, True, pa, need[0], need[4:22])
            main.wait_stream(side)
            x.record_stream(side)
            for t in [hb, bb] + [t for c in _unit_ctxs(ctx.sub_b) + [c3] for t in c.saved_tensors]:
                if isinstance(t, torch.Tensor):
                    t.record_stream(main)
        cg = _SubCtx((True, True, True, False))
        y = GateFn.forward(cg, a, bb, x, True)
        ctx.c3, ctx.cg = c3, cg
        _stash(ctx, _unit_ctxs(ctx.sub_a + ctx.sub_b) + [c3, cg])
        return y

    @staticmethod
    def backward(ctx, gy):
        with _unstash(ctx):
            da, db, gx, _ = GateFn.backward(ctx.cg, gy)
            side = ctx.side
            if side is None or _ledger.active() is not None:
                dhb, dw3, db3, _, _ = ConvFn.backward(ctx.c3, db)
                xb, flat_b = _chain_backward(ctx.sub_b, dhb, dx_res2=gx)
                dx, flat_a = _chain_backward(ctx.sub_a, da, dx_res2=xb)
            else:
                # branch b on the side stream under branch a's later units; a's first unit waits for it (its dgrad
                # epilogue adds b's input gradient)
                main = torch.cuda.current_stream(gy.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    dhb, dw3, db3, _, _ = ConvFn.backward(ctx.c3, db)
                    xb, flat_b = _chain_backward(ctx.sub_b, dhb, dx_res2=gx)
                db.record_stream(side)
                gx.record_stream(side)
                for t in [xb, dw3, db3, *flat_b]:
                    if isinstance(t, torch.Tensor):
                        t.record_stream(main)
                dx, flat_a = _chain_backward(ctx.sub_a, da, dx_res2=xb, before_first=lambda: main.wait_stream(side))
        return (dx, None, None, None, *flat_a, *flat_b, dw3, db3)


# ---------------------------------------------------------------------------
# GDN / IGDN
# ---------------------------------------------------------------------------

class GdnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, beta_raw, gamma_raw, inverse: bool, beta_min: float, reparam_offset: float):
        _check_cuda(x, beta_raw, gamma_raw)
        dt = compute_dtype()
        code = dcode(dt)
        B, C, H, W = x.shape
        xpm, xld = to_pm(x, dt, 8)
        npix = B * H * W
        st = _stream()
        br = beta_raw.detach().float().contiguous()
        gr = gamma_raw.detach().float().contiguous()
        # the model forward's pack_many launch has reparametrised this layer already (_prepack.py)
        packer = _prepack_active()
        pre = (packer.lookup(gamma_raw, dt, ("gdn", float(beta_min), float(reparam_offset)))
               if packer is not None and gr.data_ptr() == gamma_raw.data_ptr() else None)
        if pre is not None:
            beta, gop = pre
        else:
            beta = torch.empty(C, dtype=torch.float32, device=x.device)
            gop = torch.empty(2 * C * C, dtype=dt, device=x.device)
            lib.cai_gdn_reparam(_p(br), _p(gr), C, beta_min, reparam_offset, code, _p(beta), _p(gop), st)
        y = empty_pm(B, C, H, W, dt, x.device)
        _ledger.run(lambda: lib.cai_gdn_fwd(code, _p(xpm), xld, npix, C, _p(gop), _p(beta), int(inverse), _p(y), C, st),
                    "gdn_fwd", lambda: _gdn_name(code, npix, C, xld, 0), 2.0 * npix * C * C, 2 * npix * C * _es(dt) + C * C * _es(dt), dt,
                    f"{'IGDN' if inverse else 'GDN'} C={C} npix={npix}")
        ctx.save_for_backward(xpm, br, gr, beta, gop)
        ctx.cfg = (dt, xld, int(inverse), float(beta_min), float(reparam_offset))
        ctx.params = (beta_raw, gamma_raw)
        return y

    @staticmethod
    def backward(ctx, gy):
        xpm, br, gr, beta, gop = ctx.saved_tensors
        dt, xld, inverse, beta_min, off = ctx.cfg
        code = dcode(dt)
        B, C, H, W = xpm.shape
        npix = B * H * W
        st = _stream()
        gpm, gld = to_pm(gy, dt, 8)
        dx = empty_pm(B, C, H, W, dt, gy.device)
        nbytes = lib.cai_gdn_backward_workspace_bytes(npix, C, code)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=gy.device)
        bp, gp = ctx.params
        direct = direct_grad(bp) and direct_grad(gp)
        if direct:
            dbr, dgr = bp.grad, gp.grad
        else:
            dbr = torch.empty(C, dtype=torch.float32, device=gy.device)
            dgr = torch.empty((C, C), dtype=torch.float32, device=gy.device)
        if _GDN_TWO_PASS:   # A/B knob: the two-kernel path (dx + u, then the split-K parameter gradient)
            u = torch.empty(npix * C, dtype=dt, device=gy.device)
            lib.cai_gdn_bwd(code, _p(xpm), xld, _p(gpm), gld, npix, C, _p(gop), _p(beta), inverse, _p(dx), C, _p(u),
                            st)
            nb2 = lib.cai_gdn_param_grad_workspace_bytes(npix, C, code)
            ws2 = torch.empty(nb2, dtype=torch.uint8, device=gy.device)
            lib.cai_gdn_param_grad(code, _p(xpm), xld, _p(u), npix, C, _p(br), _p(gr), beta_min, off, _p(dbr),
                                   _p(dgr), int(direct), _p(ws2), nb2, st)
        elif defer_reduce_ok(direct):
            job = ReduceJob()
            lib.cai_gdn_backward_deferred(code, _p(xpm), xld, _p(gpm), gld, npix, C, _p(gop), _p(beta), inverse,
                                          _p(dx), C, _p(br), _p(gr), beta_min, off, _p(dbr), _p(dgr), 1, _p(ws),
                                          nbytes, st, ctypes.byref(job))
            defer_job(job, gy.device, ws, br, gr)
        else:
            # dx and the parameter gradients in one call (fused pass for bf16, C in {64, 128})
            _ledger.run(lambda dbr=dbr, dgr=dgr: lib.cai_gdn_backward(code, _p(xpm), xld, _p(gpm), gld, npix, C, _p(gop),
                                                                      _p(beta), inverse, _p(dx), C, _p(br), _p(gr),
                                                                      beta_min, off, _p(dbr), _p(dgr), int(direct),
                                                                      _p(ws), nbytes, st),
                        "gdn_bwd", lambda: _gdn_name(code, npix, C, max(xld, gld), 1),
                        4.0 * npix * C * C,
                        3 * npix * C * _es(dt) + 8 * C * C, dt, f"{'IGDN' if inverse else 'GDN'} C={C} npix={npix}")
        if direct:
            dbr = dgr = None
        return dx, dbr, dgr, None, None, None


class Gdn1OutFn(torch.autograd.Function):
    """GDN1 (layers/gdn.py:111-121) after its |x| 1x1 conv: y = x * (1 / norm)  (inverse: x * norm)."""

    @staticmethod
    def forward(ctx, x, norm, inverse: bool):
        _check_cuda(x, norm)
        dt = compute_dtype()
        B, C, H, W = x.shape
        xp, xld = to_pm(x, dt, _vec(dt))
        npm, nld = to_pm(norm, dt, _vec(dt))
        y, yld = _out_pm_like(x, dt)
        _ledger.run(lambda: lib.cai_gdn1_out(dcode(dt), _p(xp), xld, _p(npm), nld, _p(y), yld, B * H * W, C,
                                             int(inverse), _stream()),
                    "gdn1_out", "gdn1_out_kernel", 0, 3 * B * H * W * C * _es(dt), dt)
        ctx.save_for_backward(xp, npm)
        ctx.cfg = (dt, xld, nld, bool(inverse))
        return y

    @staticmethod
    def backward(ctx, g):
        xp, npm = ctx.saved_tensors
        dt, xld, nld, inverse = ctx.cfg
        B, C, H, W = xp.shape
        gp, gld = to_pm(g, dt, _vec(dt))
        dx, dxld = _out_pm_like(xp, dt)
        dn, dnld = _out_pm_like(xp, dt)
        _ledger.run(lambda: lib.cai_gdn1_out_bwd(dcode(dt), _p(xp), xld, _p(npm), nld, _p(gp), gld, _p(dx), dxld,
                                                 _p(dn), dnld, B * H * W, C, int(inverse), _stream()),
                    "gdn1_out_bwd", "gdn1_out_bwd_kernel", 0, 5 * B * H * W * C * _es(dt), dt)
        return dx, dn, None


# ---------------------------------------------------------------------------
# entropy models
# ---------------------------------------------------------------------------

class DeviceDraw:
    """A U(-1/2, 1/2) training-noise draw of `shape` that no kernel of its own makes and no buffer holds: the
    first entropy kernel that consumes it draws it (cai_noise_src DRAW: reads the device generator's draw index,
    records {seed, draw} in `slot`, advances the index) and every later consumer -- the other forward kernel
    sharing the draw, the backward -- regenerates it from the slot (REPLAY).  Element (p, c) equals element
    p*C + c of cai_uniform_noise's draw into a dense pixel-major buffer, so a DRAW launch reproduces a BUF
    launch fed by cai_uniform_noise bit for bit (tests/test_noise_gpu.py).  Replaces the reference's
    empty_like(x).uniform_(-0.5, 0.5) + add (entropy_models.py:170) like cai_uniform_noise, minus one launch
    and the noise tensor's write + reads per draw."""

    __slots__ = ("shape", "slot", "state", "drawn")

    def __init__(self, shape, state: torch.Tensor):
        self.shape = tuple(shape)
        self.state = state
        self.slot = torch.empty(2, dtype=torch.int64, device=state.device)
        self.drawn = False

    def record_stream(self, s):
        self.slot.record_stream(s)

    def src(self) -> NoiseSrc:
        S = NoiseSrc()
        S.kind = NOISE_REPLAY if self.drawn else NOISE_DRAW
        S.state = self.state.data_ptr()
        S.slot = self.slot.data_ptr()
        self.drawn = True
        return S


def noise_src(noise, rows: Optional[torch.Tensor] = None, ld: int = 0):
    """The cai_noise_src of a noise operand (None: no noise): a DeviceDraw, or a BUF over `rows` / ld."""
    if noise is None:
        return None
    if isinstance(noise, DeviceDraw):
        return ctypes.byref(noise.src())
    S = NoiseSrc()
    S.kind, S.ld, S.buf = NOISE_BUF, ld, rows.data_ptr()
    return ctypes.byref(S)


class GaussianFn(torch.autograd.Function):
    """GaussianConditional.forward (entropy_models.py:715-731) as one fused kernel pair."""

    @staticmethod
    def forward(ctx, x, scales, means, noise, mode: int, scale_bound: float, lik_bound: float,
                scales_relu: bool = False):
        """noise: None (DEQUANTIZE), an fp32 tensor, or a DeviceDraw.  scales_relu: the scales are a ReLU's output
        whose backward mask the caller left to this op (the producing conv ran with act_bwd_downstream)."""
        draw = noise if isinstance(noise, DeviceDraw) else None
        _check_cuda(x, scales, means, None if draw is not None else noise)
        xr, xld, npix, C = as_rows(x)
        if means is not None and means.dtype != scales.dtype:
            means = means.to(scales.dtype)
        sr, sld, _, _ = as_rows(scales)
        mr, mld = (None, 0) if means is None else as_rows(means)[:2]
        nr, nld = (None, 0) if noise is None or draw is not None else as_rows(noise)[:2]
        nsrc = noise_src(noise, nr, nld)
        smdt = dcode(scales.dtype)
        q, qbuf = empty_rows_like(x.shape, x.dtype, x.device)
        lik, lbuf = empty_rows_like(x.shape, torch.float32, x.device)
        n_el = npix * C
        _ledger.run(lambda: lib.cai_gc_fwd(mode, npix, C, _p(xr), dcode(x.dtype), xld, _p(sr), sld, _p(mr), mld, smdt,
                                           nsrc, scale_bound, lik_bound, _p(qbuf), dcode(x.dtype), C, _p(lbuf),
                                           C, _stream()),
                    "gc_fwd", "gc_fwd_kernel", 0,
                    n_el * (2 * x.element_size() + scales.element_size() * (2 if means is not None else 1) + 4
                            + (4 if nr is not None else 0)), torch.float32, f"{n_el} elements")
        ctx.save_for_backward(xr, sr, mr, nr)
        ctx.draw = draw
        ctx.relu = bool(scales_relu)
        ctx.give = _fan_role(x, "give")
        ctx.cfg = (mode, scale_bound, lik_bound, xld, sld, mld, nld, npix, C, x.shape, x.dtype, scales.shape,
                   scales.dtype, means is not None)
        # scales / means as ChunkFn's halves of one [pixels][2C] buffer: their gradients go to one such buffer too
        ctx.paired = (means is not None and scales.dim() == 4 and sld == 2 * C and mld == 2 * C
                      and means.data_ptr() == scales.data_ptr() + C * scales.element_size())
        return q, lik

    @staticmethod
    def backward(ctx, gq, glik):
        xr, sr, mr, nr = ctx.saved_tensors
        mode, sb, lb, xld, sld, mld, nld, npix, C, xshape, xdtype, sshape, sdtype, has_m = ctx.cfg
        nsrc = noise_src(ctx.draw if ctx.draw is not None else nr, nr, nld)
        gl = gq_r = None
        glld = gqld = 0
        if glik is not None:
            gl, glld = as_rows(glik.float())[:2]
        if gq is not None:
            gq_r, gqld = as_rows(gq)[:2]
        dx, dxb = empty_rows_like(xshape, xdtype, xr.device)
        dld = C
        if ctx.paired:    # both gradients in one [pixels][2C] buffer: ChunkFn's backward hands it back whole
            pair, _ = empty_rows_like((sshape[0], 2 * C, *sshape[2:]), sdtype, xr.device)
            ds = dsb = pair[:, :C]
            dm = dmb = pair[:, C:]
            dld = 2 * C
        else:
            ds, dsb = empty_rows_like(sshape, sdtype, xr.device)
            dm, dmb = empty_rows_like(sshape, sdtype, xr.device) if has_m else (None, None)
        n_el = npix * C
        es_x, es_s = xr.element_size(), sr.element_size()
        gmode = mode | (GC_SCALES_RELU if ctx.relu else 0)
        _ledger.run(lambda: lib.cai_gc_bwd(gmode, npix, C, _p(xr), dcode(xdtype), xld, _p(sr), sld, _p(mr), mld,
                                           dcode(sdtype), nsrc, sb, lb, _p(gl), glld, _p(gq_r),
                                           dcode(gq_r.dtype) if gq_r is not None else F32, gqld, _p(dxb), C, _p(dsb),
                                           dld, _p(dmb), dld, _stream()),
                    "gc_bwd", "gc_bwd_kernel", 0,
                    n_el * (2 * es_x + (4 if mr is not None else 2) * es_s + (4 if nr is not None else 0)
                            + (4 if gl is not None else 0) + (es_x if gq_r is not None else 0)),
                    torch.float32, f"{n_el} elements")
        if ctx.give is not None:    # FanOutFn: x's other consumer adds it (in its dgrad epilogue)
            ctx.give.pending, dx = dx, None
        return dx, ds, dm, None, None, None, None, None


def _eb_params(params: Sequence[torch.Tensor], quantiles: torch.Tensor) -> EbParams:
    P = EbParams()
    for i in range(5):
        P.matrix[i] = params[i].data_ptr()
        P.bias[i] = params[5 + i].data_ptr()
    for i in range(4):
        P.factor[i] = params[10 + i].data_ptr()
    P.quantiles = quantiles.data_ptr()
    return P


class BottleneckFn(torch.autograd.Function):
    """EntropyBottleneck.forward (entropy_models.py:495-540) minus the permutes."""

    @staticmethod
    def forward(ctx, x, quantiles, noise, mode: int, lik_bound: float, *params):
        """noise: None (DEQUANTIZE), an fp32 tensor, or a DeviceDraw."""
        draw = noise if isinstance(noise, DeviceDraw) else None
        _check_cuda(x, quantiles, None if draw is not None else noise)
        prm = [p.detach().float().contiguous() for p in params]
        q_ = quantiles.detach().float().contiguous()
        xr, xld, npix, C = as_rows(x)
        nr, nld = (None, 0) if noise is None or draw is not None else as_rows(noise)[:2]
        nsrc = noise_src(noise, nr, nld)
        q, qbuf = empty_rows_like(x.shape, x.dtype, x.device)
        lik, lbuf = empty_rows_like(x.shape, torch.float32, x.device)
        P = _eb_params(prm, q_)
        n_el = npix * C
        _ledger.run(lambda: lib.cai_eb_fwd(mode, npix, C, ctypes.byref(P), _p(xr), dcode(x.dtype), xld, nsrc,
                                           lik_bound, _p(qbuf), dcode(x.dtype), C, _p(lbuf), C, _stream()),
                    "eb_fwd", "eb_fwd_kernel", 0, n_el * (2 * x.element_size() + 4 + (4 if nr is not None else 0)),
                    torch.float32, f"{n_el} elements")
        ctx.save_for_backward(xr, nr, q_, *prm)
        ctx.draw = draw
        ctx.cfg = (mode, lik_bound, xld, nld, npix, C, x.shape, x.dtype)
        ctx.params = (quantiles,) + tuple(params)
        return q, lik

    @staticmethod
    def backward(ctx, gq, glik):
        xr, nr, q_, *prm = ctx.saved_tensors
        mode, lb, xld, nld, npix, C, xshape, xdtype = ctx.cfg
        nsrc = noise_src(ctx.draw if ctx.draw is not None else nr, nr, nld)
        gl = gq_r = None
        glld = gqld = 0
        if glik is not None:
            gl, glld = as_rows(glik.float())[:2]
        if gq is not None:
            gq_r, gqld = as_rows(gq)[:2]
        dx, dxb = empty_rows_like(xshape, xdtype, xr.device)
        direct = all(direct_grad(p) for p in ctx.params)
        if direct:
            dq, grads = ctx.params[0].grad, [p.grad for p in ctx.params[1:]]
        else:
            grads = [torch.empty_like(p) for p in prm]
            dq = torch.empty_like(q_)
        G = EbGrads()
        for i in range(5):
            G.matrix[i] = grads[i].data_ptr()
            G.bias[i] = grads[5 + i].data_ptr()
        for i in range(4):
            G.factor[i] = grads[10 + i].data_ptr()
        G.quantiles = dq.data_ptr()
        G.accumulate = int(direct)
        P = _eb_params(prm, q_)
        n_el = npix * C
        nsc = lib.cai_eb_scratch_bytes(npix, C)
        scratch = torch.empty(nsc, dtype=torch.uint8, device=xr.device)
        tickets = _eb_tickets(ctx.params[0], C)
        _ledger.run(lambda: lib.cai_eb_bwd(mode, npix, C, ctypes.byref(P), _p(xr), dcode(xdtype), xld, nsrc, lb,
                                           _p(gl), glld, _p(gq_r), dcode(gq_r.dtype) if gq_r is not None else F32,
                                           gqld, _p(dxb), C, ctypes.byref(G), _p(scratch), nsc, _p(tickets),
                                           _stream()),
                    "eb_bwd", "eb_bwd_kernel", 0, n_el * (3 * xr.element_size() + 8), torch.float32,
                    f"{n_el} elements")
        if direct:
            return (dx, None, None, None, None, *([None] * len(grads)))
        return (dx, dq, None, None, None, *grads)


_UNIT_GRAD = {}
_EB_TICKETS_ATTR = "_cai_eb_tickets"
_EB_AUX_SLOT = 1 << 12


def _eb_tickets(quantiles: torch.Tensor, C: int = 0, aux: bool = False) -> torch.Tensor:
    """Zeroed uint32 hand-off tickets of one EntropyBottleneck's kernels (cai_eb_bwd: one per channel;
    cai_eb_aux_loss: one, in its own slot), owned by the module's `quantiles` parameter.  Every launch leaves
    them at zero, so one buffer serves all of the module's calls and graph replays (a module's EntropyBottleneck
    launches never overlap: the forward's side stream ends before its backward, the aux loss runs after the
    backward); two models -- e.g. replicas stepped from two host threads -- never share one."""
    t = getattr(quantiles, _EB_TICKETS_ATTR, None)
    if t is None or t.device != quantiles.device:
        t = torch.zeros(_EB_AUX_SLOT + 64, dtype=torch.int32, device=quantiles.device)
        setattr(quantiles, _EB_TICKETS_ATTR, t)
    if C > _EB_AUX_SLOT:
        raise ValueError(f"EntropyBottleneck with {C} channels: at most {_EB_AUX_SLOT}")
    return t[_EB_AUX_SLOT:] if aux else t


def _unit_grad(device) -> torch.Tensor:
    """A persistent device scalar 1.0 (created once per device, outside any captured graph's steady state)."""
    t = _UNIT_GRAD.get(device)
    if t is None:
        t = torch.ones((), dtype=torch.float32, device=device)
        _UNIT_GRAD[device] = t
    return t


def loss_seed(loss: torch.Tensor):
    """The backward seed dloss/dloss = 1 of a scalar fp32 loss as a persistent device tensor (``loss.backward()``
    would fill a fresh one: one more launch in every captured step); None (the default seed) otherwise."""
    if loss.dim() == 0 and loss.dtype == torch.float32 and loss.is_cuda:
        return _unit_grad(loss.device)
    return None


class BottleneckAuxFn(torch.autograd.Function):
    """EntropyBottleneck.loss (entropy_models.py:450-454): gradient reaches only `quantiles`.

    The loss is |F(quantiles) - target| summed, so d loss / d quantiles is linear in the upstream gradient:
    the forward launch also produces it for an upstream gradient of 1, and the backward only scales it
    (one elementwise launch, cai_axpy_dev into a direct gradient, instead of a second pass through the 5-layer
    CDF chains)."""

    @staticmethod
    def forward(ctx, quantiles, target, *params):
        _check_cuda(quantiles)
        prm = [p.detach().float().contiguous() for p in params]
        q_ = quantiles.detach().float().contiguous()
        C = q_.shape[0]
        t = target.float().contiguous()
        loss = torch.empty((), dtype=torch.float32, device=quantiles.device)
        dq1 = torch.empty_like(q_)
        P = _eb_params(prm, q_)
        nsc = lib.cai_eb_scratch_bytes(0, C)
        scratch = torch.empty(nsc, dtype=torch.uint8, device=quantiles.device)
        lib.cai_eb_aux_loss(C, ctypes.byref(P), _p(t), _p(loss), _p(_unit_grad(quantiles.device)), _p(dq1), 0,
                            _p(scratch), nsc, _p(_eb_tickets(quantiles, aux=True)), _stream())
        ctx.save_for_backward(dq1)
        ctx.qparam = quantiles
        ctx.nparams = len(prm)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dq1,) = ctx.saved_tensors
        gl = g.float().reshape(())
        if direct_grad(ctx.qparam):
            gq = ctx.qparam.grad
            if not gq.is_contiguous() or gq.numel() != dq1.numel():
                raise RuntimeError("BottleneckAuxFn: a direct gradient must be a contiguous view of the flat buffer")
            _ledger.run(lambda dq1=dq1, gl=gl, gq=gq: lib.cai_axpy_dev(dq1.numel(), _p(dq1), _p(gl), _p(gq),
                                                                       _stream()),
                        "eb_aux_bwd", "axpy_dev_kernel", 0, 12 * dq1.numel(), torch.float32)
            return (None, None, *([None] * ctx.nparams))
        return ((dq1 * gl).view_as(ctx.qparam), None, *([None] * ctx.nparams))


# ---------------------------------------------------------------------------
# rate-distortion loss (examples/train.py:68-82)
# ---------------------------------------------------------------------------

class RdLossFnUnfused(torch.autograd.Function):
    """The per-tensor reduction path (cai_sum_log / cai_sum_sqdiff + torch scalar ops): A/B reference."""

    @staticmethod
    def forward(ctx, x_hat, target, lmbda: float, npix: int, *liks):
        _check_cuda(x_hat, target, *liks)
        xh = x_hat.float().contiguous()
        tg = target.float().contiguous()
        n = xh.numel()
        st = _stream()
        sums = torch.empty(len(liks) + 1, dtype=torch.float32, device=xh.device)
        rows = []
        for i, l in enumerate(liks):
            lr, ld, lp, C = as_rows(l.float())
            rows.append((lr, ld, lp, C))
            nb = lib.cai_reduce_workspace_bytes(lp * C)
            ws = torch.empty(nb, dtype=torch.uint8, device=xh.device)
            lib.cai_sum_log(_p(lr), lp, C, ld, _p(sums[i:i + 1]), _p(ws), nb, st)
        nb = lib.cai_reduce_workspace_bytes(n)
        ws = torch.empty(nb, dtype=torch.uint8, device=xh.device)
        lib.cai_sum_sqdiff(_p(xh), _p(tg), n, _p(sums[-1:]), _p(ws), nb, st)
        bpp_coef = 1.0 / (-math.log(2) * npix)
        bpp = sums[:-1].sum() * bpp_coef
        mse = sums[-1] / n
        loss = lmbda * mse + bpp
        ctx.save_for_backward(xh, tg, *[r[0] for r in rows])
        ctx.cfg = (lmbda, bpp_coef, n, [(r[1], r[2], r[3]) for r in rows], [l.shape for l in liks], x_hat.shape)
        return loss, mse, bpp

    @staticmethod
    def backward(ctx, gl, gm, gb):
        xh, tg, *lrs = ctx.saved_tensors
        lmbda, bpp_coef, n, meta, lshapes, xshape = ctx.cfg
        zero = torch.zeros((), dtype=torch.float32, device=xh.device)
        gl = zero if gl is None else gl.float()
        gm = zero if gm is None else gm.float()
        gb = zero if gb is None else gb.float()
        gbt = (gb + gl).reshape(1).contiguous()
        gmt = (gm + lmbda * gl).reshape(1).contiguous()
        st = _stream()
        dxh = torch.empty_like(xh)
        lib.cai_sqdiff_bwd(_p(xh), _p(tg), n, _p(gmt), 2.0 / n, _p(dxh), st)
        dliks = []
        for lr, (ld, lp, C), shp in zip(lrs, meta, lshapes):
            d, dbuf = empty_rows_like(shp, torch.float32, xh.device)
            lib.cai_log_bwd(_p(lr), lp, C, ld, _p(gbt), bpp_coef, _p(dbuf), st)
            dliks.append(d)
        return (dxh.view(xshape), None, None, None, *dliks)


class RdLossFn(torch.autograd.Function):
    """RateDistortionLoss (examples/train.py:68-82): forward in two launches (cai_rd_loss_fwd), backward in
    one (cai_rd_loss_bwd); the upstream gradients stay on the device."""

    @staticmethod
    def forward(ctx, x_hat, target, lmbda: float, npix: int, *liks):
        _check_cuda(x_hat, target, *liks)
        if not 1 <= len(liks) <= 4:
            raise ValueError("RD loss takes 1 to 4 likelihood tensors")
        xh = x_hat.float().contiguous()
        tg = target.float().contiguous()
        if xh.shape != tg.shape:
            raise ValueError(f"x_hat {tuple(xh.shape)} and target {tuple(tg.shape)} differ")
        lbufs = []
        for l in liks:
            r, ld, lp, C = as_rows(l.float())
            if ld != C:
                r = r.contiguous() if r.is_contiguous() else l.float().contiguous()
            lbufs.append(r)
        bpp_coef = 1.0 / (-math.log(2) * npix)
        desc = RdInputs()
        for i, r in enumerate(lbufs):
            desc.lik[i] = r.data_ptr()
            desc.lik_n[i] = r.numel()
        desc.nlik, desc.x_hat, desc.target, desc.n = len(lbufs), xh.data_ptr(), tg.data_ptr(), xh.numel()
        out = torch.empty(3, dtype=torch.float32, device=xh.device)
        ws = torch.empty(lib.cai_rd_loss_workspace_bytes(), dtype=torch.uint8, device=xh.device)
        nl = sum(r.numel() for r in lbufs)
        _ledger.run(lambda: lib.cai_rd_loss_fwd(ctypes.byref(desc), float(lmbda), bpp_coef, _p(out), _p(ws),
                                                ws.numel(), _stream()),
                    "rd_fwd", "rd_stage1/2", 0, 8 * xh.numel() + 4 * nl, torch.float32)
        ctx.save_for_backward(xh, tg, *lbufs)
        ctx.cfg = (float(lmbda), bpp_coef, [l.shape for l in liks], x_hat.shape)
        # unused outputs (mse, bpp when only the loss is backpropagated) reach backward as None, not as
        # zero-filled tensors (two fill launches per step); the kernel reads a null gradient as 0
        ctx.set_materialize_grads(False)
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, gl, gm, gb):
        xh, tg, *lbufs = ctx.saved_tensors
        lmbda, bpp_coef, lshapes, xshape = ctx.cfg
        desc = RdInputs()
        grads = RdGrads()
        dliks = []
        for i, (r, shp) in enumerate(zip(lbufs, lshapes)):
            desc.lik[i] = r.data_ptr()
            desc.lik_n[i] = r.numel()
            d = torch.empty_like(r)
            grads.dlik[i] = d.data_ptr()
            dliks.append(d)
        desc.nlik, desc.x_hat, desc.target, desc.n = len(lbufs), xh.data_ptr(), tg.data_ptr(), xh.numel()
        dxh = torch.empty_like(xh)
        g = [None if t is None else t.float().contiguous() for t in (gl, gm, gb)]
        nl = sum(r.numel() for r in lbufs)
        _ledger.run(lambda: lib.cai_rd_loss_bwd(ctypes.byref(desc), lmbda, bpp_coef, _p(g[0]), _p(g[1]), _p(g[2]),
                                                _p(dxh), ctypes.byref(grads), _stream()),
                    "rd_bwd", "rd_bwd_kernel", 0, 12 * xh.numel() + 8 * nl, torch.float32)
        # each likelihood gradient in the layout of its buffer, viewed with the logical shape
        outs = []
        for d, r, shp in zip(dliks, lbufs, lshapes):
            outs.append(_like_logical(d, r, shp))
        return (dxh.view(xshape), None, None, None, *outs)


def _like_logical(d: torch.Tensor, buf: torch.Tensor, shape) -> torch.Tensor:
    """d has buf's memory layout; return it as a tensor of the likelihood's logical shape."""
    if tuple(buf.shape) == tuple(shape):
        return d.as_strided(buf.shape, buf.stride())
    # as_rows moved the channel dim last: [B, *spatial, C] -> logical [B, C, *spatial]
    return d.movedim(-1, 1)


# ---------------------------------------------------------------------------
# pointwise glue of the residual / attention / sub-pixel blocks
# (layers/layers.py:81-244) -- csrc/elementwise.hip
# ---------------------------------------------------------------------------

def _out_pm_like(t: torch.Tensor, dtype) -> Tuple[torch.Tensor, int]:
    B, C, H, W = t.shape
    ld = (C + _vec(dtype) - 1) // _vec(dtype) * _vec(dtype)
    return empty_pm(B, C, H, W, dtype, t.device, ld=ld), ld


_MASK_OF_ACT = {ACT_RELU: MASK_POS, ACT_LEAKY: MASK_LEAKY}


def _act_grad(g, y, ld_y, act, prm, dtype):
    """g * act'(pre) from the activated output y (y > 0 <=> pre > 0 for ReLU / LeakyReLU)."""
    gp, gld = to_pm(g, dtype, _vec(dtype))
    if act == ACT_NONE:
        return gp
    out, old = _out_pm_like(g, dtype)
    B, C, H, W = g.shape
    _ledger.run(lambda: lib.cai_act_bwd(_MASK_OF_ACT[act], prm, _p(y), ld_y, _p(gp), gld, _p(out), old, B * H * W, C,
                                        dcode(dtype), _stream()),
                "act_bwd", "act_bwd_kernel", 0, 3 * B * H * W * C * _es(dtype), dtype)
    return out


class AddActFn(torch.autograd.Function):
    """y = act(a + b): the residual `out += identity` (+ the trailing ReLU of ResidualUnit)."""

    @staticmethod
    def forward(ctx, a, b, act: int, prm: float):
        _check_cuda(a, b)
        if a.shape != b.shape:
            raise ValueError(f"residual add: shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
        dt = compute_dtype()
        vec = _vec(dt)
        ap, ald = to_pm(a, dt, vec)
        bp, bld = to_pm(b, dt, vec)
        y, yld = _out_pm_like(a, dt)
        B, C, H, W = a.shape
        _ledger.run(lambda: lib.cai_add_act(dcode(dt), _p(ap), ald, _p(bp), bld, _p(y), yld, B * H * W, C, act, prm,
                                            _stream()),
                    "add_act", "add_act_kernel", 0, 3 * B * H * W * C * _es(dt), dt)
        ctx.cfg = (act, prm, dt, yld)
        ctx.save_for_backward(y if act != ACT_NONE else None)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        act, prm, dt, yld = ctx.cfg
        d = _act_grad(g, y, yld, act, prm, dt)
        return d, d, None, None


class ActFn(torch.autograd.Function):
    """Standalone ReLU / LeakyReLU (when no conv epilogue can absorb it)."""

    @staticmethod
    def forward(ctx, x, act: int, prm: float):
        _check_cuda(x)
        dt = compute_dtype()
        xp, xld = to_pm(x, dt, _vec(dt))
        y, yld = _out_pm_like(x, dt)
        B, C, H, W = x.shape
        lib.cai_act(dcode(dt), _p(xp), xld, _p(y), yld, B * H * W, C, act, prm, _stream())
        ctx.cfg = (act, prm, dt, yld)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        act, prm, dt, yld = ctx.cfg
        return _act_grad(g, y, yld, act, prm, dt), None, None


class GateFn(torch.autograd.Function):
    """AttentionBlock (layers.py:238-243): y = a * sigmoid(b) + x.  relu_a: a is a ReLU output whose producer
    (ResidualChainFn with out_masked) expects its gradient already masked: da carries the mask."""

    @staticmethod
    def forward(ctx, a, b, x, relu_a: bool = False):
        _check_cuda(a, b, x)
        dt = compute_dtype()
        B, C, H, W = a.shape
        ld = (C + _vec(dt) - 1) // _vec(dt) * _vec(dt)

        def same(t):   # the kernel takes one ld for a, b, x, y
            tp, tld = to_pm(t, dt, _vec(dt))
            if tld != ld:
                tp2 = empty_pm(B, C, H, W, dt, t.device, ld=ld)
                tp2.copy_(tp)
                tp = tp2
            return tp
        ap, bp, xp = same(a), same(b), same(x)
        y = empty_pm(B, C, H, W, dt, a.device, ld=ld)
        _ledger.run(lambda: lib.cai_gate_fwd(dcode(dt), _p(ap), _p(bp), _p(xp), _p(y), ld, B * H * W, C, _stream()),
                    "gate_fwd", "gate_fwd_kernel", 0, 4 * B * H * W * C * _es(dt), dt)
        ctx.cfg = (dt, ld, int(relu_a))
        ctx.save_for_backward(ap, bp)
        return y

    @staticmethod
    def backward(ctx, g):
        ap, bp = ctx.saved_tensors
        dt, ld, relu_a = ctx.cfg
        B, C, H, W = ap.shape
        gp, gld = to_pm(g, dt, _vec(dt))
        da = empty_pm(B, C, H, W, dt, g.device, ld=ld)
        db = empty_pm(B, C, H, W, dt, g.device, ld=ld)
        _ledger.run(lambda: lib.cai_gate_bwd(dcode(dt), _p(ap), _p(bp), _p(gp), gld, _p(da), _p(db), ld, B * H * W, C,
                                             relu_a, _stream()),
                    "gate_bwd", "gate_bwd_kernel", 0, 5 * B * H * W * C * _es(dt), dt)
        return da, db, g, None


def _bhwc_strides(t: torch.Tensor):
    s = t.stride()
    return (ctypes.c_int64 * 4)(s[0], s[2], s[3], s[1])


class PixelShuffleFn(torch.autograd.Function):
    """nn.PixelShuffle(r) (subpel_conv3x3, layers.py:86-91) on any layout; pixel-major stays pixel-major."""

    @staticmethod
    def forward(ctx, x, r: int):
        _check_cuda(x)
        B, Cr, H, W = x.shape
        if Cr % (r * r):
            raise ValueError(f"pixel_shuffle: {Cr} channels not divisible by r^2 = {r * r}")
        C = Cr // (r * r)
        dt = x.dtype
        if dt not in (torch.float32, torch.bfloat16):
            raise ValueError("pixel_shuffle: fp32 / bf16 only")
        pm = pixel_major_ld(x) is not None and C % _vec(dt) == 0
        y = empty_pm(B, C, H * r, W * r, dt, x.device) if pm else torch.empty((B, C, H * r, W * r), dtype=dt,
                                                                              device=x.device)
        lib.cai_pixel_shuffle(dcode(dt), _p(x), _bhwc_strides(x), _p(y), _bhwc_strides(y), B, H, W, C, r, 0,
                              _stream())
        ctx.cfg = (r, dt, tuple(x.shape), pixel_major_ld(x) is not None)
        return y

    @staticmethod
    def backward(ctx, g):
        r, dt, xshape, x_pm = ctx.cfg
        B, Cr, H, W = xshape
        g = g.to(dt)
        dx = empty_pm(B, Cr, H, W, dt, g.device) if x_pm else torch.empty(xshape, dtype=dt, device=g.device)
        lib.cai_pixel_shuffle(dcode(dt), _p(g), _bhwc_strides(g), _p(dx), _bhwc_strides(dx), B, H, W, Cr // (r * r),
                              r, 1, _stream())
        return dx, None


# ---------------------------------------------------------------------------
# multi-modal codec alignment modules (models/master.py) -- csrc/swin.hip.
# Token sequences (B, L, C) are held as pixel-major [B, C, Hr, Wr] tensors:
# row b*L + l, exactly the reference's flattened token order.
# ---------------------------------------------------------------------------

class CatFn(torch.autograd.Function):
    """torch.cat(tensors, dim=1) into one pixel-major buffer (HIP copies); grads are channel views."""

    @staticmethod
    def forward(ctx, *ts):
        _check_cuda(*ts)
        dt = compute_dtype()
        vec = _vec(dt)
        B, _, H, W = ts[0].shape
        cs = [t.shape[1] for t in ts]
        if any(c % vec for c in cs[:-1]):
            raise ValueError("cat: leading channel counts must be multiples of the vector width")
        total = sum(cs)
        ld = (total + vec - 1) // vec * vec
        out = empty_pm(B, total, H, W, dt, ts[0].device, ld=ld)
        off = 0
        for t, c in zip(ts, cs):
            tp, tld = to_pm(t, dt, vec)
            dst = _VP(out.data_ptr() + off * out.element_size())
            lib.cai_act(dcode(dt), _p(tp), tld, dst, ld, B * H * W, c, ACT_NONE, 0.0, _stream())
            off += c
        ctx.cs = cs
        return out

    @staticmethod
    def backward(ctx, g):
        outs, off = [], 0
        for c in ctx.cs:
            outs.append(g[:, off:off + c])
            off += c
        return tuple(outs)


class ChunkFn(torch.autograd.Function):
    """t.chunk(2, 1) for the entropy parameters' (scales, means) pair (models/google.py): channel views forward.
    Backward: when GaussianFn wrote both gradients into one [pixels][2C] buffer (the pair's halves, adjacent), that
    buffer IS t's gradient -- handed back as it is, no concatenation; otherwise the halves are copied natively into
    one pixel-major buffer (torch's chunk backward is an ATen cat)."""

    @staticmethod
    def forward(ctx, t):
        C = t.shape[1] // 2
        ctx.cfg = (C, tuple(t.shape))
        return t[:, :C], t[:, C:]

    @staticmethod
    def backward(ctx, gs, gm):
        C, shape = ctx.cfg
        if (gs is not None and gm is not None and gs.dtype == gm.dtype and gs.stride() == gm.stride()
                and pixel_major_ld(gs) == 2 * C and gm.data_ptr() == gs.data_ptr() + C * gs.element_size()):
            return gs.as_strided(shape, gs.stride())
        ref = gs if gs is not None else gm
        dt = ref.dtype
        B, _, H, W = shape
        out = empty_pm(B, 2 * C, H, W, dt, ref.device, ld=2 * C)
        for k, g in enumerate((gs, gm)):
            if g is None:
                g = torch.zeros((B, C, H, W), dtype=dt, device=ref.device)
            gp, gld = to_pm(g.to(dt), dt, _vec(dt))
            dst = _VP(out.data_ptr() + k * C * out.element_size())
            lib.cai_act(dcode(dt), _p(gp), gld, dst, 2 * C, B * H * W, C, ACT_NONE, 0.0, _stream())
        return out


class LayerNormFn(torch.autograd.Function):
    """nn.LayerNorm(C) over the channel dim of pixel-major tokens."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps: float):
        _check_cuda(x, weight, bias)
        dt = compute_dtype()
        B, C, H, W = x.shape
        xp, xld = to_pm(x, dt, _vec(dt))
        y, yld = _out_pm_like(x, dt)
        n = B * H * W
        mean = torch.empty(n, dtype=torch.float32, device=x.device)
        rstd = torch.empty(n, dtype=torch.float32, device=x.device)
        w = weight.detach().float().contiguous()
        lib.cai_layernorm_fwd(dcode(dt), _p(xp), xld, n, C, _p(w), _p(bias.detach().float().contiguous()), eps,
                              _p(y), yld, _p(mean), _p(rstd), _stream())
        ctx.save_for_backward(xp, w, mean, rstd)
        ctx.cfg = (dt, xld)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, g):
        xp, w, mean, rstd = ctx.saved_tensors
        dt, xld = ctx.cfg
        B, C, H, W = xp.shape
        n = B * H * W
        gp, gld = to_pm(g, dt, _vec(dt))
        dx, dxld = _out_pm_like(xp, dt)
        wparam, bparam = ctx.params
        direct = direct_grad(wparam) and direct_grad(bparam)
        dw = wparam.grad if direct else torch.empty(C, dtype=torch.float32, device=g.device)
        db = bparam.grad if direct else torch.empty(C, dtype=torch.float32, device=g.device)
        nb = lib.cai_layernorm_bwd_workspace_bytes(n, C)
        ws = torch.empty(nb, dtype=torch.uint8, device=g.device)
        lib.cai_layernorm_bwd(dcode(dt), _p(xp), xld, _p(gp), gld, n, C, _p(w), _p(mean), _p(rstd), _p(dx), dxld,
                              _p(dw), _p(db), int(direct), _p(ws), nb, _stream())
        if direct:
            return dx, None, None, None
        return dx, dw, db, None


class GeluFn(torch.autograd.Function):
    """nn.GELU() (exact erf form)."""

    @staticmethod
    def forward(ctx, x):
        _check_cuda(x)
        dt = compute_dtype()
        B, C, H, W = x.shape
        xp, xld = to_pm(x, dt, _vec(dt))
        y, yld = _out_pm_like(x, dt)
        lib.cai_gelu_fwd(dcode(dt), _p(xp), xld, _p(y), yld, B * H * W, C, _stream())
        ctx.save_for_backward(xp)
        ctx.cfg = (dt, xld)
        return y

    @staticmethod
    def backward(ctx, g):
        (xp,) = ctx.saved_tensors
        dt, xld = ctx.cfg
        B, C, H, W = xp.shape
        gp, gld = to_pm(g, dt, _vec(dt))
        dx, dxld = _out_pm_like(xp, dt)
        lib.cai_gelu_bwd(dcode(dt), _p(xp), xld, _p(gp), gld, _p(dx), dxld, B * H * W, C, _stream())
        return dx


class WindowAttnFn(torch.autograd.Function):
    """WindowAttention core (master.py:534-566, before proj) with the block's shift / partition folded in."""

    @staticmethod
    def forward(ctx, q, kv, table, rel_index, mask, cfg):
        _check_cuda(q, kv, table)
        dt = compute_dtype()
        (Hr, Wr, heads, window, shift, scale) = cfg
        B, C, H, W = q.shape
        if H * W != Hr * Wr:
            raise ValueError(f"window attention: {H * W} tokens for a {Hr}x{Wr} resolution")
        qp, qld = to_pm(q, dt, _vec(dt))
        kp, kld = to_pm(kv, dt, _vec(dt))
        tb = table.detach().float().contiguous()
        P = _attn_desc(qp, qld, kp, kld, tb, rel_index, mask, B, Hr, Wr, heads, window, shift, scale)
        out, old = _out_pm_like(q, dt)
        lib.cai_window_attn_fwd(dcode(dt), ctypes.byref(P), _p(out), old, _stream())
        ctx.save_for_backward(qp, kp, tb)
        ctx.cfg = (dt, qld, kld, rel_index, mask, B, Hr, Wr, heads, window, shift, scale)
        ctx.tparam = table
        return out

    @staticmethod
    def backward(ctx, g):
        qp, kp, tb = ctx.saved_tensors
        dt, qld, kld, rel_index, mask, B, Hr, Wr, heads, window, shift, scale = ctx.cfg
        P = _attn_desc(qp, qld, kp, kld, tb, rel_index, mask, B, Hr, Wr, heads, window, shift, scale)
        gp, gld = to_pm(g, dt, _vec(dt))
        dq, dqld = _out_pm_like(qp, dt)
        dkv, dkvld = _out_pm_like(kp, dt)
        direct = direct_grad(ctx.tparam)
        dtab = ctx.tparam.grad if direct else torch.empty(tb.shape, dtype=torch.float32, device=g.device)
        nb = lib.cai_window_attn_bwd_workspace_bytes(ctypes.byref(P))
        ws = torch.empty(nb, dtype=torch.uint8, device=g.device)
        lib.cai_window_attn_bwd(dcode(dt), ctypes.byref(P), _p(gp), gld, _p(dq), dqld, _p(dkv), dkvld, _p(dtab),
                                int(direct), _p(ws), nb, _stream())
        return dq, dkv, (None if direct else dtab), None, None, None


def _attn_desc(qp, qld, kp, kld, tb, rel_index, mask, B, Hr, Wr, heads, window, shift, scale):
    from ._native import WindowAttn

    return WindowAttn(_VP(qp.data_ptr()), qld, _VP(kp.data_ptr()), kld, _VP(tb.data_ptr()),
                      _VP(rel_index.data_ptr()), _VP(mask.data_ptr()) if mask is not None else None, B, Hr, Wr,
                      heads, qp.shape[1] // heads, window, shift, scale)


def _mean_ws(B, HW, C, device):
    nb = lib.cai_channel_mean_workspace_bytes(B, HW, C)
    return torch.empty(max(nb, 16), dtype=torch.uint8, device=device), nb


class ChannelMeanFn(torch.autograd.Function):
    """nn.AdaptiveAvgPool2d(1) of a pixel-major map -> [B, C, 1, 1] fp32."""

    @staticmethod
    def forward(ctx, x):
        _check_cuda(x)
        dt = compute_dtype()
        B, C, H, W = x.shape
        xp, xld = to_pm(x, dt, _vec(dt))
        out = torch.empty((B, C, 1, 1), dtype=torch.float32, device=x.device)
        ws, nb = _mean_ws(B, H * W, C, x.device)
        lib.cai_channel_mean(dcode(dt), _p(xp), xld, None, 0, B, H * W, C, _p(out), 1.0 / (H * W), _p(ws), nb,
                             _stream())
        ctx.cfg = (dt, tuple(x.shape))
        return out

    @staticmethod
    def backward(ctx, g):
        dt, (B, C, H, W) = ctx.cfg
        gb = g.float().contiguous()
        dx = empty_pm(B, C, H, W, dt, g.device, ld=(C + _vec(dt) - 1) // _vec(dt) * _vec(dt))
        lib.cai_channel_affine(dcode(dt), None, 0, None, _p(gb), 1.0 / (H * W), _p(dx), pixel_major_ld(dx), B, H * W,
                               C, _stream())
        return dx


class ChannelAffineFn(torch.autograd.Function):
    """gamma * x + beta with per-(image, channel) gamma / beta [B, C, 1, 1] (Channel_aligner output)."""

    @staticmethod
    def forward(ctx, x, gamma, beta):
        _check_cuda(x, gamma, beta)
        dt = compute_dtype()
        B, C, H, W = x.shape
        xp, xld = to_pm(x, dt, _vec(dt))
        ga, be = gamma.float().contiguous(), beta.float().contiguous()
        y, yld = _out_pm_like(x, dt)
        lib.cai_channel_affine(dcode(dt), _p(xp), xld, _p(ga), _p(be), 1.0, _p(y), yld, B, H * W, C, _stream())
        ctx.save_for_backward(xp, ga)
        ctx.cfg = (dt, xld)
        return y

    @staticmethod
    def backward(ctx, g):
        xp, ga = ctx.saved_tensors
        dt, xld = ctx.cfg
        B, C, H, W = xp.shape
        gp, gld = to_pm(g, dt, _vec(dt))
        dx, dxld = _out_pm_like(xp, dt)
        lib.cai_channel_affine(dcode(dt), _p(gp), gld, _p(ga), None, 0.0, _p(dx), dxld, B, H * W, C, _stream())
        dgamma = torch.empty((B, C, 1, 1), dtype=torch.float32, device=g.device)
        dbeta = torch.empty((B, C, 1, 1), dtype=torch.float32, device=g.device)
        ws, nb = _mean_ws(B, H * W, C, g.device)
        lib.cai_channel_mean(dcode(dt), _p(gp), gld, _p(xp), xld, B, H * W, C, _p(dgamma), 1.0, _p(ws), nb, _stream())
        lib.cai_channel_mean(dcode(dt), _p(gp), gld, None, 0, B, H * W, C, _p(dbeta), 1.0, _p(ws), nb, _stream())
        return dx, dgamma, dbeta
