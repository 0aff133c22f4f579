"""Fused Adam over one flat fp32 parameter buffer (examples/train.py:111-142,176-186).

``FusedAdam(params, lr, betas, eps)`` behaves like ``torch.optim.Adam`` (no
weight decay, no amsgrad): the parameters are re-homed as views of a single
flat buffer and their ``.grad`` as views of a flat gradient buffer (autograd
accumulates into it in place), so one ``cai_adam`` launch updates everything
and ``step(max_norm=...)`` folds ``clip_grad_norm_`` in: the squared norm is a
deterministic device reduction and the clip coefficient is applied inside the
Adam kernel -- no host synchronisation, so a whole training step can be
captured in one HIP graph.  The flat gradient is also the single buffer the
data-parallel all-reduce runs on (compressai.distributed).
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Optional, Tuple

import torch

from ._native import lib
from ._ops import DIRECT_GRAD_ATTR, _p, _stream


def _align(n: int, a: int = 4) -> int:
    return (n + a - 1) // a * a


class FusedAdam:
    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8):
        self.params: List[torch.nn.Parameter] = [p for p in params]
        if not self.params:
            raise ValueError("optimizer got an empty parameter list")
        dev = self.params[0].device
        if dev.type != "cuda":
            raise ValueError("FusedAdam runs on GPU parameters only")
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        offs, n = [], 0
        for p in self.params:
            if p.dtype != torch.float32:
                raise ValueError("FusedAdam expects fp32 master parameters")
            offs.append(n)
            n += _align(p.numel())
        self.numel = n
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_count = torch.zeros(1, dtype=torch.float32, device=dev)
        self.sqnorm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = torch.empty(lib.cai_reduce_workspace_bytes(n), dtype=torch.uint8, device=dev)
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                view = self.flat[o:o + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
                p.grad = self.flat_grad[o:o + p.numel()].view_as(p)
                # let the backward kernels accumulate into p.grad directly
                setattr(p, DIRECT_GRAD_ATTR, True)

    def zero_grad(self, set_to_none: bool = False):
        # grads stay views of the flat buffer (set_to_none is ignored on purpose)
        self.flat_grad.zero_()

    def grad_sqnorm(self) -> torch.Tensor:
        lib.cai_sqnorm(_p(self.flat_grad), self.numel, _p(self.sqnorm), _p(self._ws), self._ws.numel(), _stream())
        return self.sqnorm

    def step(self, max_norm: Optional[float] = None):
        sq = None
        if max_norm is not None and max_norm > 0:
            self.grad_sqnorm()
            sq = self.sqnorm
        lib.cai_adam(_p(self.flat), _p(self.flat_grad), _p(self.exp_avg), _p(self.exp_avg_sq), self.numel, self.lr,
                     self.betas[0], self.betas[1], self.eps, _p(self.step_count), _p(sq),
                     float(max_norm) if sq is not None else 0.0, _stream())

    def state_dict(self):
        return {"lr": self.lr, "betas": self.betas, "eps": self.eps, "step": self.step_count.clone(),
                "exp_avg": self.exp_avg.clone(), "exp_avg_sq": self.exp_avg_sq.clone()}

    def load_state_dict(self, sd):
        self.lr, self.betas, self.eps = sd["lr"], tuple(sd["betas"]), sd["eps"]
        self.step_count.copy_(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])


def parameter_groups(net):
    """train.py:115-124: names of the main (all but `.quantiles`) and aux (`.quantiles`) parameters, sorted."""
    named = dict(net.named_parameters())
    main = sorted(n for n, p in named.items() if not n.endswith(".quantiles") and p.requires_grad)
    aux = sorted(n for n, p in named.items() if n.endswith(".quantiles") and p.requires_grad)
    assert len(set(main) & set(aux)) == 0 and len(set(main) | set(aux)) == len(named)
    return main, aux


def configure_optimizers(net, lr: float = 1e-4, aux_lr: float = 1e-3):
    """train.py:111-142: main Adam on all but `.quantiles`, aux Adam on `.quantiles` (sorted by name)."""
    named = dict(net.named_parameters())
    main, aux = parameter_groups(net)
    return FusedAdam((named[n] for n in main), lr=lr), FusedAdam((named[n] for n in aux), lr=aux_lr)
