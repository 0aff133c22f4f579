"""Fused Adam over one flat fp32 parameter buffer (examples/train.py:111-142,176-186).

``FusedAdam(params, lr, betas, eps)`` is a ``torch.optim.Optimizer`` with
``torch.optim.Adam`` semantics (no weight decay, no amsgrad), so the
reference's callers work on it unchanged: ``GradScaler.unscale_/step``,
``clip_grad_norm_``, ``StepLR`` (it reads ``param_groups[0]["lr"]`` at every
``step``) and ``state_dict()`` / ``load_state_dict()`` in torch's per-parameter
Adam format (train.py:407,419,475).

The parameters are re-homed as views of a single flat buffer and their
``.grad`` as views of a flat gradient buffer (autograd and the backward
kernels accumulate into it in place), so one ``cai_adam`` launch updates
everything and ``step(max_norm=...)`` folds ``clip_grad_norm_`` in: the squared
norm is a deterministic device reduction and the clip coefficient is applied
inside the Adam kernel -- no host synchronisation, so a whole training step can
be captured in one HIP graph.  A non-finite gradient norm skips the update on
the device (GradScaler's skip rule).  The flat gradient is also the single
buffer the data-parallel all-reduce runs on (compressai.distributed).

If a caller breaks the gradient views (``model.zero_grad()`` with torch's
default ``set_to_none=True``, or ``p.grad = None``), ``step`` copies the fresh
gradients back into the flat buffer and re-attaches the views, so no update
ever runs on stale gradients.
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional, Tuple

import torch

from . import _ledger
from ._native import ADAM_CLIP, ADAM_SKIP_NONFINITE, ADAM_SMALL_N, ADAM_ZERO_GRAD, lib
from ._ops import DIRECT_GRAD_ATTR, _p, _stream


def _align(n: int, a: int = 4) -> int:
    return (n + a - 1) // a * a


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, skip_nonfinite: bool = True, layout: Optional[List[int]] = None,
                 zero_grad_in_step: bool = False):
        """layout: optional permutation of the parameter indices giving their order in the flat buffers
        (param_groups / state_dict keep the given order); distributed.OverlappedAllReduce puts the
        parameters whose gradients finish last at the end so the rest can be exchanged early.

        zero_grad_in_step: step() consumes the gradients (the Adam kernel zeroes each one as it reads it)
        and zero_grad() right after a step() launches nothing.  For the reference's loop order
        (zero_grad, forward, backward, step: train.py:172-186); p.grad reads zero after step()."""
        params = [p for p in params]
        if not params:
            raise ValueError("optimizer got an empty parameter list")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"Invalid beta parameters: {betas}")
        super().__init__(params, dict(lr=float(lr), betas=(float(betas[0]), float(betas[1])), eps=float(eps)))
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdam takes one parameter group")
        self.params: List[torch.nn.Parameter] = list(self.param_groups[0]["params"])
        dev = self.params[0].device
        if dev.type != "cuda":
            raise ValueError("FusedAdam runs on GPU parameters only")
        self.skip_nonfinite = bool(skip_nonfinite)
        self.zero_grad_in_step = bool(zero_grad_in_step)
        self._grads_consumed = False
        order = list(range(len(self.params))) if layout is None else [int(i) for i in layout]
        if sorted(order) != list(range(len(self.params))):
            raise ValueError("layout must be a permutation of the parameter indices")
        offs, n = [0] * len(self.params), 0
        for i in order:
            p = self.params[i]
            if p.dtype != torch.float32:
                raise ValueError("FusedAdam expects fp32 master parameters")
            if p.device != dev:
                raise ValueError("FusedAdam expects all parameters on one device")
            offs[i] = n
            n += _align(p.numel())
        self.offsets = offs
        self.numel = n
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_count = torch.zeros(1, dtype=torch.float32, device=dev)
        self.sqnorm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = torch.empty(max(lib.cai_reduce_workspace_bytes(n), lib.cai_adam_step_workspace_bytes(n)),
                               dtype=torch.uint8, device=dev)
        self._grad_views = []
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                view = self.flat[o:o + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
                self._grad_views.append(self.flat_grad[o:o + p.numel()].view_as(p))
                # let the backward kernels accumulate into p.grad directly
                setattr(p, DIRECT_GRAD_ATTR, True)
        self._attach_views()

    # -- compatibility knobs read by older callers -------------------------------------------------
    @property
    def lr(self) -> float:
        return float(self.param_groups[0]["lr"])

    @lr.setter
    def lr(self, v: float):
        self.param_groups[0]["lr"] = float(v)

    @property
    def betas(self) -> Tuple[float, float]:
        return tuple(self.param_groups[0]["betas"])

    @property
    def eps(self) -> float:
        return float(self.param_groups[0]["eps"])

    # -- gradient views ------------------------------------------------------------------------------
    def _attach_views(self):
        for p, v in zip(self.params, self._grad_views):
            p.grad = v

    def _sync_grad_views(self):
        """Re-home gradients a caller detached from the flat buffer (host-side pointer check; launches
        only when a view was actually broken)."""
        for p, v in zip(self.params, self._grad_views):
            g = p.grad
            if g is None:
                v.zero_()
            elif g.data_ptr() != v.data_ptr() or g.shape != v.shape:
                v.copy_(g)
            else:
                continue
            p.grad = v

    def zero_grad(self, set_to_none: bool = True):
        # the gradients stay views of the flat buffer; set_to_none zeroes them instead of unlinking them.
        # Right after a consuming step() they are zero already.
        if not self._grads_consumed:
            self.flat_grad.zero_()
        self._grads_consumed = False
        self._attach_views()

    def grad_sqnorm(self) -> torch.Tensor:
        _ledger.run(lambda: lib.cai_sqnorm(_p(self.flat_grad), self.numel, _p(self.sqnorm), _p(self._ws),
                                           self._ws.numel(), _stream()),
                    "sqnorm", "sqnorm (reduce)", 2.0 * self.numel, 4 * self.numel, torch.float32)
        return self.sqnorm

    @torch.no_grad()
    def step(self, closure=None, max_norm: Optional[float] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._sync_grad_views()
        clip = max_norm is not None and max_norm > 0
        flags = (ADAM_CLIP if clip else 0) | (ADAM_SKIP_NONFINITE if self.skip_nonfinite else 0)
        zero = self.zero_grad_in_step and (flags or self.numel <= ADAM_SMALL_N)
        flags |= ADAM_ZERO_GRAD if zero else 0
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        # norm + clip + Adam + step count in 2 launches (1 for small buffers): cai_adam_step; self.sqnorm
        # receives sum(g^2) whenever it is computed
        small = self.numel <= ADAM_SMALL_N
        _ledger.run(lambda: lib.cai_adam_step(_p(self.flat), _p(self.flat_grad), _p(self.exp_avg),
                                              _p(self.exp_avg_sq), self.numel, float(g["lr"]), float(b1), float(b2),
                                              float(g["eps"]), _p(self.step_count), _p(self.sqnorm),
                                              float(max_norm) if clip else math.inf, flags, _p(self._ws),
                                              self._ws.numel(), _stream()),
                    "adam", "adam_small_kernel" if small else "sq_part + adam_fused_kernel", 2.0 * self.numel if flags
                    else 0.0, 32 * self.numel if flags else 28 * self.numel, torch.float32,
                    f"{self.numel} parameters")
        self._grads_consumed = zero
        return loss

    # -- checkpoints in torch.optim.Adam's format (train.py:407,419,475) -------------------------------
    def state_dict(self):
        steps = float(self.step_count.item())
        state = {}
        if steps > 0:
            for i, (p, o) in enumerate(zip(self.params, self.offsets)):
                n = p.numel()
                state[i] = {"step": torch.tensor(steps),
                            "exp_avg": self.exp_avg[o:o + n].view_as(p).clone(),
                            "exp_avg_sq": self.exp_avg_sq[o:o + n].view_as(p).clone()}
        g = self.param_groups[0]
        group = {"lr": g["lr"], "betas": tuple(g["betas"]), "eps": g["eps"], "weight_decay": 0, "amsgrad": False,
                 "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "params": list(range(len(self.params)))}
        if "initial_lr" in g:
            group["initial_lr"] = g["initial_lr"]
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        if "exp_avg" in sd and "state" not in sd:    # the flat layout of round-1 checkpoints
            self.param_groups[0].update(lr=float(sd["lr"]), betas=tuple(sd["betas"]), eps=float(sd["eps"]))
            self.step_count.copy_(sd["step"])
            self.exp_avg.copy_(sd["exp_avg"])
            self.exp_avg_sq.copy_(sd["exp_avg_sq"])
            return
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.params):
            raise ValueError("loaded state dict does not match this optimizer's parameters")
        if groups[0].get("weight_decay", 0) or groups[0].get("amsgrad", False) or groups[0].get("maximize", False):
            raise ValueError("FusedAdam supports Adam without weight decay, amsgrad or maximize")
        g = self.param_groups[0]
        for k in ("lr", "eps", "initial_lr"):
            if k in groups[0]:
                g[k] = float(groups[0][k])
        g["betas"] = tuple(float(b) for b in groups[0]["betas"])
        state = sd["state"]
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        steps = 0.0
        for slot, pid in enumerate(groups[0]["params"]):
            s = state.get(pid)
            if not s:
                continue
            p, o = self.params[slot], self.offsets[slot]
            n = p.numel()
            if s["exp_avg"].numel() != n:
                raise ValueError(f"state of parameter {pid}: {s['exp_avg'].numel()} elements, expected {n}")
            self.exp_avg[o:o + n].copy_(s["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
            steps = float(s["step"])
        self.step_count.fill_(steps)


def parameter_groups(net):
    """train.py:115-124: names of the main (all but `.quantiles`) and aux (`.quantiles`) parameters, sorted."""
    named = dict(net.named_parameters())
    main = sorted(n for n, p in named.items() if not n.endswith(".quantiles") and p.requires_grad)
    aux = sorted(n for n, p in named.items() if n.endswith(".quantiles") and p.requires_grad)
    assert len(set(main) & set(aux)) == 0 and len(set(main) | set(aux)) == len(named)
    return main, aux


def check_tail_cuts(cuts: Tuple[str, ...]) -> Tuple[str, ...]:
    """Cuts must be listed in the order the backward reaches them: cuts of one parent in strictly
    descending child index ("g_a.4", "g_a.2").  OverlappedAllReduce.backward_phase(i) stops at cuts[i]; an
    ascending list would run phase 1 through the lower cut and leave the later phases nothing to propagate
    (silently zero gradients), so it is rejected."""
    cuts = tuple(cuts)
    last = {}
    for c in cuts:
        parent, sep, idx = c.rpartition(".")
        if not sep or not idx.isdigit():
            raise ValueError(f"tail cut {c!r}: expected '<parent>.<child index>'")
        if parent in last and int(idx) >= last[parent]:
            raise ValueError(f"tail cuts {cuts}: cuts of {parent!r} must be listed in strictly descending child "
                             f"order (the order the backward reaches them); {c!r} follows {parent}.{last[parent]}")
        last[parent] = int(idx)
    return cuts


def dp_stage(name: str, tail: Tuple[str, ...], cuts: Tuple[str, ...] = ()) -> int:
    """Gradient bucket of parameter `name` (compressai.distributed.OverlappedAllReduce): 0 outside the tail;
    in the tail 1 + the number of `cuts` ("g_a.4": the input of child 4 of the tail Sequential g_a) the
    parameter lies below, i.e. the order in which the backward finishes the buckets."""
    if not any(name.startswith(t) for t in tail):
        return 0
    below = 0
    for c in cuts:
        parent, idx = c.rsplit(".", 1)
        if name.startswith(parent + "."):
            child = name[len(parent) + 1:].split(".", 1)[0]
            if child.isdigit() and int(child) < int(idx):
                below += 1
    return 1 + below


def phase_of(name: str, plan) -> int:
    """Gradient bucket of parameter `name` under a phase plan (CompressionModel.dp_phases(): (prefixes, roots,
    inputs) per phase): the first phase one of whose prefixes `name` starts with, else the plan's catch-all
    phase (prefixes None)."""
    rest = None
    for k, (prefixes, _, _) in enumerate(plan):
        if prefixes is None:
            rest = k if rest is None else rest
        elif any(name.startswith(p) for p in prefixes):
            return k
    if rest is None:
        raise ValueError(f"parameter {name!r} belongs to no phase of the plan (and no phase takes the rest)")
    return rest


def configure_optimizers(net, lr: float = 1e-4, aux_lr: float = 1e-3, tail: Tuple[str, ...] = (),
                         zero_grad_in_step: bool = False, tail_cuts: Tuple[str, ...] = (), phases=None):
    """train.py:111-142: main Adam on all but `.quantiles`, aux Adam on `.quantiles` (sorted by name).

    tail: name prefixes whose parameters go last in the main flat buffers (FusedAdam layout); tail_cuts split
    the tail further (dp_stage): the buffer holds the buckets in backward order, head first.  The optimizer's
    ``bucket_bounds`` are the buckets' element offsets ([0, ..., numel]); ``tail_offset`` is where the tail
    starts (distributed.OverlappedAllReduce).
    phases: a phase plan (CompressionModel.dp_phases()) instead: one bucket per phase, in phase order
    (distributed.OverlappedAllReduce.for_model reads it back from ``opt.dp_plan``).
    zero_grad_in_step: see FusedAdam (both optimizers)."""
    named = dict(net.named_parameters())
    main, aux = parameter_groups(net)
    if phases is not None:
        phases = [(None if p is None else tuple(p), tuple(r), tuple(i)) for p, r, i in phases]
        stage = [phase_of(n, phases) for n in main]
        nst = len(phases)
    else:
        tail_cuts = check_tail_cuts(tail_cuts)
        stage = [dp_stage(n, tail, tail_cuts) for n in main]
        nst = 1 + len(tail_cuts) + 1 if tail else 1
    layout = [i for s in range(nst) for i, t in enumerate(stage) if t == s]
    opt = FusedAdam((named[n] for n in main), lr=lr, layout=layout, zero_grad_in_step=zero_grad_in_step)
    bounds = [0]
    for s in range(1, nst):
        offs = [opt.offsets[i] for i, t in enumerate(stage) if t >= s]
        bounds.append(min(offs) if offs else opt.numel)
    bounds.append(opt.numel)
    opt.bucket_bounds = bounds
    opt.tail_offset = bounds[1] if len(bounds) > 2 else opt.numel
    opt.dp_plan = phases
    return opt, FusedAdam((named[n] for n in aux), lr=aux_lr, zero_grad_in_step=zero_grad_in_step)
