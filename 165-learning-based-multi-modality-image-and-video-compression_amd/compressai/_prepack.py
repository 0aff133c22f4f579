"""Per-model weight packing in one launch.

Every conv needs its fp32 torch weight re-laid out (and cast) into the MFMA
layout for the forward and the input-gradient directions.  Done per call that
is ~2 small launches per conv per step (~300 for cheng2020).  A model instead
owns a ``Prepacker``: persistent packed buffers for all of its convs and a
device-resident descriptor table, refreshed by ONE ``cai_conv_pack_many``
launch at the start of every model forward (so it is inside the captured HIP
graph, after the previous optimizer step).  ConvFn looks its packed weights up
here while that forward is active and falls back to packing per call
otherwise (modules used on their own, tests).
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict, Optional, Tuple

import torch

from . import _ledger
from ._native import ConvGeom, lib
from ._ops import _p, _stream, compute_dtype, conv_geom, dcode, edge_eligible

_active = threading.local()


def active() -> Optional["Prepacker"]:
    return getattr(_active, "packer", None)


class Prepacker:
    def __init__(self, model: torch.nn.Module):
        self.model = model
        self._plans: Dict[torch.dtype, dict] = {}

    # ------------------------------------------------------------------ build
    def _convs(self):
        from .layers.conv import _ConvMixin
        from .layers.layers import MaskedConv2d

        for m in self.model.modules():
            if not isinstance(m, _ConvMixin):
                continue
            transposed = isinstance(m, torch.nn.ConvTranspose2d)
            spec = m._spec()
            if transposed and m.out_channels <= 16 and not edge_eligible(spec.k, spec.s, spec.p, m.in_channels,
                                                                         m.out_channels, transposed):
                continue   # few-channel deconv path packs its own per-pixel GEMM weights
            mask = m.mask if isinstance(m, MaskedConv2d) else None
            yield m, mask

    def _gdns(self):
        from .layers.gdn import GDN

        return [m for m in self.model.modules() if isinstance(m, GDN)]

    def _signature(self):
        return (tuple((m.weight.data_ptr(), None if k is None else k.data_ptr()) for m, k in self._convs()) +
                tuple((m.beta.data_ptr(), m.gamma.data_ptr()) for m in self._gdns()))

    def _build(self, dtype):
        dev = next(self.model.parameters()).device
        dsz = lib.cai_conv_pack_desc_bytes()
        descs, table, buffers = [], {}, []
        for m, mask in self._convs():
            spec = m._spec()
            g = conv_geom(spec, 1, m.in_channels, 16, 16, m.out_channels)   # packing ignores spatial size
            w = m.weight.detach()
            if w.dtype != torch.float32 or not w.is_contiguous():
                return None   # packing reads the fp32 master weights in place
            if edge_eligible(spec.k, spec.s, spec.p, m.in_channels, m.out_channels, spec.transposed):
                # csrc/edge.hip MFMA fragments (bf16 only): forward, and the deconv's input gradient
                if dtype != torch.bfloat16:
                    continue
                ge = conv_geom(spec, 1, m.in_channels, 32, 32, m.out_channels)
                for direction in ((0, 1) if spec.transposed else (0,)):
                    nbytes = lib.cai_edge_frag_bytes(ctypes.byref(ge), dcode(dtype), direction)
                    if nbytes == 0:
                        break
                    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
                    d = ctypes.create_string_buffer(dsz)
                    lib.cai_edge_pack_describe(ctypes.byref(ge), dcode(dtype), direction, _p(w), _p(buf), d)
                    descs.append(d.raw)
                    buffers.append(buf)
                    table[(w.data_ptr(), ("edge", direction))] = buf
                continue
            for direction in (0, 1):
                nbytes = lib.cai_conv_packed_weight_bytes(ctypes.byref(g), dcode(dtype), direction)
                buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
                d = ctypes.create_string_buffer(dsz)
                lib.cai_conv_pack_describe(ctypes.byref(g), dcode(dtype), direction, _p(w),
                                           _p(mask) if mask is not None else None, _p(buf), d)
                descs.append(d.raw)
                buffers.append(buf)
                table[(w.data_ptr(), direction)] = buf
        # GDN / IGDN reparametrisations (beta, gamma operand) in the same launch (an older library without the
        # entry point, as in A/B runs, leaves them to GdnFn)
        try:
            lib.cai_gdn_reparam_describe
            gdns = self._gdns()
        except AttributeError:
            gdns = []
        for m in gdns:
            br, gr = m.beta.detach(), m.gamma.detach()
            if br.dtype != torch.float32 or gr.dtype != torch.float32 or not (br.is_contiguous() and gr.is_contiguous()):
                continue   # GdnFn reparametrises this layer itself
            C = br.numel()
            beta = torch.empty(C, dtype=torch.float32, device=dev)
            gop = torch.empty(2 * C * C, dtype=dtype, device=dev)
            d = ctypes.create_string_buffer(dsz)
            lib.cai_gdn_reparam_describe(_p(br), _p(gr), C, float(m.beta_reparam.minimum),
                                         float(m.beta_reparam.reparam_offset), _p(beta), _p(gop), d)
            descs.append(d.raw)
            buffers += [beta, gop]
            table[(gr.data_ptr(), ("gdn", float(m.beta_reparam.minimum), float(m.beta_reparam.reparam_offset)))] = (
                beta, gop)
        if not descs:
            return None
        host = ctypes.create_string_buffer(b"".join(descs), len(descs) * dsz)
        total = lib.cai_conv_pack_finalize(host, len(descs))
        blob = torch.frombuffer(bytearray(host.raw), dtype=torch.uint8).to(dev)
        # algorithmic bytes of one pack launch (ledger): every packed buffer written once, and every fp32 source
        # (weight, mask, GDN parameters) read once -- a weight's two directions share the source tiles
        written = sum(b.numel() * b.element_size() for b in buffers)
        read = sum(4 * (m.weight.numel() + (k.numel() if k is not None else 0)) for m, k in self._convs())
        read += sum(4 * (m.beta.numel() + m.gamma.numel()) for m in gdns)
        return {"sig": self._signature(), "table": table, "buffers": buffers, "descs": blob, "n": len(descs),
                "total": total, "bytes": written + read}

    # -------------------------------------------------------------------- use
    def refresh(self):
        """Pack every conv weight of the model for the current compute dtype (one launch)."""
        dtype = compute_dtype()
        plan = self._plans.get(dtype)
        if plan is None or plan["sig"] != self._signature():
            plan = self._build(dtype)
            if plan is None:
                return None
            self._plans[dtype] = plan
        _ledger.run(lambda: lib.cai_conv_pack_many(_p(plan["descs"]), plan["n"], dcode(dtype), plan["total"], _stream()),
                    "pack", "pack_many_kernel", 0, plan.get("bytes", 0), dtype, f"{plan['n']} descriptors")
        return plan

    def lookup(self, weight: torch.Tensor, dtype, direction: int) -> Optional[torch.Tensor]:
        plan = self._plans.get(dtype)
        if plan is None:
            return None
        return plan["table"].get((weight.data_ptr(), direction))


class prepacked_forward:
    """Context of one model forward: refresh the packs, expose them to ConvFn."""

    def __init__(self, model):
        self.model = model

    def __enter__(self):
        self.prev = active()
        packer = getattr(self.model, "_cai_prepacker", None)
        if packer is None:
            packer = Prepacker(self.model)
            object.__setattr__(self.model, "_cai_prepacker", packer)
        if any(p.is_cuda for p in self.model.parameters()) and packer.refresh() is not None:
            _active.packer = packer
        else:
            _active.packer = None
        return self

    def __exit__(self, *exc):
        _active.packer = self.prev
        return False
