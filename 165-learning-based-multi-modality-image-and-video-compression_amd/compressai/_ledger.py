"""Per-launch ledger of one training step (measurement only; bench.py, tools/).

While ``recording()`` is active, every instrumented library call of
``compressai._ops`` / ``compressai.optim`` is bracketed by two HIP events on
the current stream and logged with its algorithmic work: FLOPs (MFMA-shaped
work: convolutions, the GDN 1x1 contractions) and the minimum HBM bytes
(read every operand once, write every result once).  ``SURVEY.md §8(d)``'s
whole-step roofline is the sum over entries of max(FLOP / P_mfma, bytes /
BW_hbm); the entry with the largest measured time is the step's dominant
launch.  Each entry keeps a ``replay`` closure that re-issues the same call, so
one launch can be timed (or profiled with rocprofv3) in isolation.

Outside ``recording()`` the instrumented calls cost one global lookup.
"""
from __future__ import annotations

import contextlib
from typing import Callable, List, Optional

import torch

BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
F32_PEAK_TFLOPS = 157.3     # MI355X dense fp32 MFMA
HBM_PEAK_GBS = 8000.0

_active: Optional["Ledger"] = None


class Entry:
    __slots__ = ("kind", "kernel", "flops", "nbytes", "dtype", "shape", "ev0", "ev1", "replay", "ms")

    def __init__(self, kind, kernel, flops, nbytes, dtype, shape, replay):
        self.kind, self.kernel, self.flops, self.nbytes = kind, kernel, float(flops), float(nbytes)
        self.dtype, self.shape, self.replay = dtype, shape, replay
        self.ev0 = torch.cuda.Event(enable_timing=True)
        self.ev1 = torch.cuda.Event(enable_timing=True)
        self.ms = None

    def peak_tflops(self) -> float:
        return BF16_PEAK_TFLOPS if self.dtype == torch.bfloat16 else F32_PEAK_TFLOPS

    def roofline_ms(self) -> float:
        return max(self.flops / (self.peak_tflops() * 1e9), self.nbytes / (HBM_PEAK_GBS * 1e6))

    def bound(self) -> str:
        return "mfma" if self.flops / (self.peak_tflops() * 1e9) >= self.nbytes / (HBM_PEAK_GBS * 1e6) else "hbm"

    def as_dict(self):
        d = {"kind": self.kind, "kernel": self.kernel, "shape": self.shape, "ms": self.ms,
             "flops": self.flops, "bytes": self.nbytes, "bound": self.bound(), "roofline_ms": self.roofline_ms()}
        if self.ms:
            d["tflops"] = self.flops / (self.ms * 1e9)
            d["gbs"] = self.nbytes / (self.ms * 1e6)
            d["frac"] = self.roofline_ms() / self.ms
        return d


class Ledger:
    def __init__(self, keep_replay: bool = True):
        self.entries: List[Entry] = []
        self.keep_replay = keep_replay

    def finish(self):
        torch.cuda.synchronize()
        for e in self.entries:
            e.ms = e.ev0.elapsed_time(e.ev1)
        return self


def active() -> Optional[Ledger]:
    return _active


@contextlib.contextmanager
def recording(keep_replay: bool = True):
    global _active
    prev, _active = _active, Ledger(keep_replay)
    led = _active
    try:
        yield led
    finally:
        _active = prev


def run(launch: Callable[[], object], kind: str, kernel, flops: float, nbytes: float, dtype, shape=None):
    """Issue `launch()`; inside recording() bracket it with events and log it.  `kernel` may be a
    zero-argument callable (evaluated only while recording)."""
    led = _active
    if led is None:
        return launch()
    e = Entry(kind, kernel() if callable(kernel) else kernel, flops, nbytes, dtype, shape,
              launch if led.keep_replay else None)
    e.ev0.record()
    out = launch()
    e.ev1.record()
    led.entries.append(e)
    return out


# ---------------------------------------------------------------------------------------------------------
# algorithmic work of the instrumented ops
# ---------------------------------------------------------------------------------------------------------

def conv_cost(g, es: int, direction: int, x_bytes: Optional[int] = None, y_bytes: Optional[int] = None):
    """(FLOPs, bytes) of one conv call.  direction 0 fwd, 1 input gradient, 2 weight gradient.
    MACs = B x (pixels of the stride-1 side) x Cin x Cout x k^2 for every direction; bytes = each operand
    once (activations at `es` bytes unless x_bytes / y_bytes override: the fp32 NCHW image of the edge
    layers; weights in the compute dtype, weight gradients fp32 read-modify-write)."""
    small = (g.in_h * g.in_w) if g.transposed else (g.out_h * g.out_w)
    macs = g.batch * small * g.in_c * g.out_c * g.kernel * g.kernel
    xb = (x_bytes if x_bytes is not None else es) * g.batch * g.in_h * g.in_w * g.in_c
    yb = (y_bytes if y_bytes is not None else es) * g.batch * g.out_h * g.out_w * g.out_c
    wel = g.in_c * g.out_c * g.kernel * g.kernel
    if direction == 2:
        nbytes = xb + yb + 8 * wel
    else:
        nbytes = xb + yb + es * wel
    return 2.0 * macs, float(nbytes)


def shape_of(g) -> str:
    kind = "ConvT" if g.transposed else "Conv"
    return (f"{kind} {g.in_c}->{g.out_c} k{g.kernel} s{g.stride} {g.in_h}x{g.in_w}->{g.out_h}x{g.out_w} "
            f"B={g.batch}")
