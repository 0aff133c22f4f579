"""Data parallelism: one process per GPU, gradient all-reduce over RCCL/xGMI.

The reference trains with single-process nn.DataParallel
(examples/train.py:101-108,413); here each rank owns a GPU, processes its own
patches, and the only exchange per step is the all-reduce (average) of the
flat gradient buffer of FusedAdam (20.3 MB fp32 for bmshj2018-hyperprior).
The aux loss (EntropyBottleneck.loss) depends only on replicated parameters,
so its gradients are identical on every rank and need no exchange.

OverlappedAllReduce splits that exchange in two buckets at a CUT of the
model's graph: a set of tensors through which every path from the "tail"
parameters to the loss runs.  Once the backward has reached the cut, every
other ("head") gradient is final, so that bucket is all-reduced on a side
stream while the tail's backward runs; the tail bucket follows.  The zoo
models cut at y = g_a(x) (tail: g_a); Master_compresser cuts at its feature
encoder / channel-aligner outputs (x_feature, guided_align -- the aligner is
~70 % of the step's FLOPs; guided_align also feeds fdecoder, so g_a's output
alone is not a cut).  Models declare their tail as ``dp_tail`` (parameter
name prefixes) and mark the cut in forward with ``self._dp_cut(...)``
(models/google.py CompressionModel).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend: str = None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def allreduce_mean_(flat: torch.Tensor):
    """In-place mean over ranks of one flat buffer (RCCL ncclAvg on GPU, SUM/world on gloo)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return flat
    if dist.get_backend() == "nccl":
        dist.all_reduce(flat, op=dist.ReduceOp.AVG)
    else:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.div_(dist.get_world_size())
    return flat


def broadcast_parameters_(module: torch.nn.Module, src: int = 0):
    """Make every rank start from rank src's weights."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    for t in list(module.parameters()) + list(module.buffers()):
        if t.numel():
            dist.broadcast(t.data, src)



class _Boundary(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g


def _cut_site(model: torch.nn.Module, name: str):
    """Where cut `name` is marked: "<seq>.<k>" (the input of child k, "g_a.4") in the parent's cut slot for a
    product Sequential (compressai.layers.Sequential), else by the child's forward pre-hook; any other name
    by the model's own forward (_dp_mark)."""
    from .layers.conv import Sequential

    parent, sep, idx = name.rpartition(".")
    if not sep or not idx.isdigit():
        return model
    pm = model.get_submodule(parent)
    if isinstance(pm, Sequential):
        return (pm, int(idx))
    return _PreCut(model.get_submodule(name))


class _PreCut:
    """A forward pre-hook site (the input of a module that is not a product Sequential's child)."""

    def __init__(self, module):
        self.module = module

    def register_forward_pre_hook(self, fn):
        return self.module.register_forward_pre_hook(fn)


class OverlappedAllReduce:
    """Bucketed gradient all-reduce overlapped with the backward.

    The backward runs as a sequence of PHASES, one per gradient bucket, in the order the backward finishes
    them.  Phase i is ``torch.autograd.backward(roots_i, inputs=[*cuts_i, *params_i])``: it propagates the
    gradients of its root cuts (phase 0: the loss) down to its input cuts -- identity boundary nodes the
    forward inserted at named points of the graph -- and no further, so bucket i (params_i, contiguous in
    FusedAdam's flat gradient buffer) is final when it ends.  ``reduce_bucket(i)`` all-reduces bucket i on a
    side stream while phase i + 1 runs on the compute stream; ``finish()`` all-reduces the last bucket and
    joins the streams.  Each phase can be captured in its own HIP graph; the collectives stay outside the
    graphs (stream order only, no events).  ``backward_head(loss)`` is phase 0, ``backward_phase(i)`` the
    others; ``reduce_head()`` / ``backward_tail()`` are the eager form.

    The plan -- ``phases``: a list of (params, roots, inputs), cut NAMES in roots / inputs -- comes from the
    model (``CompressionModel.dp_phases()``: e.g. cheng2020-attn: g_s in three pieces, the context /
    entropy-parameter stack, the hyper path, then g_a in four pieces).  A cut named "<seq>.<k>" is the input of
    child k of a Sequential (its cut slot, or a forward pre-hook); any other name is a point the model's forward
    marks itself with ``_dp_mark(name, *tensors)``.  Each cut is the input of exactly one phase and a root of
    exactly one later phase: its gradient is held from the one to the other.  A phase with no inputs (the last) differentiates everything below its roots.
    No input of a phase may lie below another of its inputs: autograd would run the path between them to
    complete the lower one (the context phase therefore stops at "yq" -- y as quantize and the
    GaussianConditional read it -- not at y, which the hyper path below its "params" cut also reaches).

    Legacy form (positional ``split, tail, head_params, cut_modules, stage_params``): the head, then a tail
    (a model with a ``_dp_cut`` marker, or a module whose output is the cut) cut further at the inputs of
    ``cut_modules``.

    Cut tensors accumulate over the grad-enabled forwards of a step (micro-batches summed into one loss) and
    are released by ``finish()``; a plain ``loss.backward()`` outside the phases (no exchange) releases the
    ones it differentiated through, so they never leak into the next step.  The cuts of a grad-enabled
    forward the step's loss does not depend on (one computed for logging, never backpropagated) are dropped
    by ``backward_head`` (a reachability walk from the loss, only when more than one forward marked a cut).

    Memory: each phase keeps the graph (retain_graph) because the later phases still need its saved
    tensors; they are released when the caller drops its loss tensor (bench.py's step drops it on return) --
    the serial backward's peak otherwise."""

    def __init__(self, flat_grad: torch.Tensor, split, tail=None, head_params=(), cut_modules=(),
                 stage_params=None, phases=None, sites=None):
        bounds = list(split) if isinstance(split, (list, tuple)) else [0, int(split), flat_grad.numel()]
        self._model = None
        self._handles = []
        self._slots = []
        if phases is None:
            # legacy: head -> "y" (the tail's output) -> "cut1" ... (inputs of cut_modules) -> input
            if len(bounds) != len(cut_modules) + 3 and not (len(bounds) == 2 and not cut_modules):
                raise ValueError("OverlappedAllReduce: one bucket per cut piece expected "
                                 f"({len(cut_modules) + 2} buckets for {len(cut_modules)} tail cuts, bounds {bounds})")
            names = ["y"] + [f"cut{k}" for k in range(1, len(cut_modules) + 1)]
            phases = [(list(head_params), ["loss"], names[:1])]
            for k in range(len(cut_modules) + 1):
                ps = (stage_params or [])[k] if k < len(stage_params or []) else []
                phases.append((list(ps), [names[k]], names[k + 1:k + 2]))
            if len(bounds) == 2:            # one bucket: one phase, the whole backward
                phases, names = [(list(head_params), ["loss"], [])], []
            sites = {"y": tail}
            sites.update({f"cut{k + 1}": m for k, m in enumerate(cut_modules)})
        if len(bounds) != len(phases) + 1:
            raise ValueError(f"OverlappedAllReduce: {len(phases)} phases need {len(phases) + 1} bucket bounds, "
                             f"got {bounds}")
        self.buckets = [flat_grad[bounds[i]:bounds[i + 1]] for i in range(len(bounds) - 1)]
        self.head = self.buckets[0]
        self.tail = flat_grad[bounds[1]:] if len(bounds) > 2 else flat_grad[:0]
        self.phases = [([p for p in ps if p.requires_grad], list(r), list(i)) for ps, r, i in phases]
        self.head_params = self.phases[0][0]
        # (a CPU buffer -- the gloo tests of the phase logic -- reduces synchronously, no side stream)
        self.side = torch.cuda.Stream(device=flat_grad.device) if flat_grad.is_cuda else None
        self._names = sorted({n for _, r, i in self.phases for n in (*r, *i) if n != "loss"})
        self._first = self.phases[0][2][0] if self.phases[0][2] else None   # the cut every forward reaches
        self._cuts = {n: [] for n in self._names}
        self._grads = {}                # id(cut tensor) -> its gradient, from its input phase to its root phase
        for n in self._names:           # a cut is the input of one phase and the root of a later one
            ins = [k for k, (_, _, inp) in enumerate(self.phases) if n in inp]
            outs = [k for k, (_, r, _) in enumerate(self.phases) if n in r]
            if len(ins) != 1 or len(outs) != 1 or not ins[0] < outs[0]:
                raise ValueError(f"OverlappedAllReduce: cut {n!r} must be the input of one phase and the root of a "
                                 f"later one (inputs of phases {ins}, roots of phases {outs})")
        self._in_phase = False
        self._nfwd = 0                  # grad-enabled forwards that marked the first cut since the last step
        for n in self._names:
            self._attach(n, (sites or {}).get(n))

    def _attach(self, name, site):
        """Insert the boundary of cut `name` at its site: a model's own marks (_dp_mark / _dp_cut), a product
        Sequential's cut slot, a forward pre-hook (the input of a module) or a forward hook (a module's output)."""
        if site is None:
            return
        if isinstance(site, tuple):
            # (parent Sequential, child index): the product Sequential runs its children through .run()
            # (conv + activation epilogue fusion), so the cut goes into its own cut slots
            parent, idx = site
            parent.__dict__.setdefault("_cut_fns", {})[idx] = lambda x, n=name: self._mark(n, x)[0]
            self._slots.append((parent, idx))
        elif isinstance(site, _PreCut) or name.startswith("cut"):
            mod = site.module if isinstance(site, _PreCut) else site
            self._handles.append(mod.register_forward_pre_hook(
                lambda m, inputs, n=name: (self._mark(n, inputs[0])[0],) + tuple(inputs[1:])))
        elif hasattr(site, "_dp_mark"):
            self._model = site
            site._dp_mark_fn = lambda n, *ts: self._mark(n, *ts)
        elif hasattr(site, "_dp_cut") and hasattr(site, "dp_tail"):
            self._model = site
            site._dp_cut_fn = lambda *ts, n=name: self._mark(n, *ts)
        else:
            # a module whose output is the cut (e.g. net.g_a of the zoo models)
            self._handles.append(site.register_forward_hook(lambda m, i, o, n=name: self._mark(n, o)[0]))

    @classmethod
    def for_model(cls, model: torch.nn.Module, opt):
        """The exchange of `model` over FusedAdam `opt` built by configure_optimizers(model,
        phases=model.dp_phases()) (one bucket per phase); a buffer built with the legacy tail / tail_cuts
        arguments gets the legacy phases."""
        from .optim import check_tail_cuts, dp_stage, phase_of

        bounds = list(getattr(opt, "bucket_bounds", [0, opt.tail_offset, opt.numel]))
        main = [(n, p) for n, p in model.named_parameters() if not n.endswith(".quantiles")]
        plan = getattr(opt, "dp_plan", None)
        if plan is not None:
            stage = [phase_of(n, plan) for n, _ in main]
            phases = [([p for (n, p), s in zip(main, stage) if s == k], r, i) for k, (_, r, i) in enumerate(plan)]
            names = {n for _, r, i in plan for n in (*r, *i) if n != "loss"}
            return cls(opt.flat_grad, bounds, phases=phases, sites={n: _cut_site(model, n) for n in names})
        tail = tuple(model.dp_tail)
        cuts = check_tail_cuts(getattr(model, "dp_tail_cuts", ())) if len(bounds) > 3 else ()
        head = [p for n, p in main if dp_stage(n, tail, cuts) == 0]
        stages = [[p for n, p in main if dp_stage(n, tail, cuts) == s] for s in range(1, len(cuts) + 2)]
        return cls(opt.flat_grad, bounds, model, head, [_cut_site(model, c) for c in cuts], stages)

    @property
    def nphases(self) -> int:
        return len(self.buckets)

    def _mark(self, name, *ts):
        # only a forward that can be differentiated marks its cut (no_grad / eval passes go through as is), and
        # only the cuts of this exchange's plan (a model marks every point it knows)
        if name not in self._cuts or not torch.is_grad_enabled() or not any(t.requires_grad for t in ts):
            return ts
        # boundary nodes: a phase's capture of a cut tensor's gradient may execute its grad_fn, which for
        # the product convs writes parameter gradients as a side effect; an identity node in between has none
        out = tuple(_Boundary.apply(t) for t in ts)
        if name == self._first:
            self._nfwd += 1
        for t in out:
            # a backward outside the phases (a plain loss.backward()) releases the cut (by id: a reference in the
            # hook would keep the tensor, and with it its graph, alive until the cycle collector runs)
            t.register_hook(lambda g, tid=id(t), n=name: self._release(n, tid))
        self._cuts[name].extend(out)
        return out

    def _release(self, name, tid):
        if not self._in_phase:
            self._cuts[name] = [c for c in self._cuts[name] if id(c) != tid]
            if name == self._first and not self._cuts[name]:
                self._nfwd = 0
        return None

    def _prune(self, loss: torch.Tensor):
        """Drop the cut tensors of grad-enabled forwards this loss does not depend on (a forward computed for
        logging and never backpropagated): they would keep their graphs alive for the step and be passed to
        the phases as inputs.  Only needed when more than one forward marked its cut since the last step."""
        if self._nfwd <= 1:
            return
        seen, stack = set(), [loss.grad_fn]
        while stack:
            n = stack.pop()
            if n is None or n in seen:
                continue
            seen.add(n)
            stack.extend(f for f, _ in n.next_functions)
        self._cuts = {k: [t for t in c if t.grad_fn in seen] for k, c in self._cuts.items()}
        self._nfwd = 1

    def _backward(self, roots, grads, i: int):
        """Phase i: differentiate `roots` down to its input cuts and bucket parameters.  The cuts' gradients come
        back from torch.autograd.grad and are kept here (``self._grads``) as the next phases' seeds: routing
        them through .grad would copy each into the tensor's layout and, once a cut is a root, add its own seed
        to it again (ATen copy + add launches over the 67 MB activations of the 128x128 maps)."""
        params, _, names = self.phases[i]
        cuts = [t for n in names for t in self._cuts[n]]
        self._in_phase = True
        try:
            if not cuts and i == self.nphases - 1:
                torch.autograd.backward(roots, grad_tensors=grads)      # the last phase: everything below
                return
            inputs = cuts + params
            outs = torch.autograd.grad(roots, inputs, grad_outputs=grads, retain_graph=True, allow_unused=True)
        finally:
            self._in_phase = False
        for t, g in zip(cuts, outs[:len(cuts)]):
            if g is not None:
                self._grads[id(t)] = g
        for p, g in zip(params, outs[len(cuts):]):
            # the product kernels write straight into the flat buffer (direct_grad) and return no gradient; an
            # op that returns one accumulates it as backward() would
            if g is not None:
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.add_(g)

    def backward_head(self, loss: torch.Tensor):
        self._prune(loss)
        if self._first is not None and not self._cuts[self._first]:
            raise RuntimeError("OverlappedAllReduce: the forward did not reach the cut")
        from ._ops import loss_seed

        self._grads = {}
        # retain_graph: the engine releases the saved tensors of every node of the graph it was given,
        # including the later phases', which they still need
        self._backward([loss], [loss_seed(loss)], 0)

    def backward_phase(self, i: int):
        """Phase i (1 .. nphases - 1): from its root cuts' gradients down to its input cuts."""
        ys = [y for n in self.phases[i][1] for y in self._cuts[n] if id(y) in self._grads]
        if ys:
            self._backward(ys, [self._grads.pop(id(y)) for y in ys], i)

    def reduce_bucket(self, i: int):
        """All-reduce bucket i on the side stream, after everything queued on the compute stream."""
        if self.side is None:
            if self.buckets[i].numel():
                allreduce_mean_(self.buckets[i])
            return
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            if self.buckets[i].numel():
                allreduce_mean_(self.buckets[i])

    def reduce_head(self):
        self.reduce_bucket(0)

    def backward_tail(self):
        """Every later phase, eagerly: bucket i is all-reduced while phase i + 1 runs (the last by finish())."""
        for i in range(1, self.nphases):
            self.backward_phase(i)
            if i < self.nphases - 1:
                self.reduce_bucket(i)

    def finish(self):
        """All-reduce the last bucket after the whole backward, join the side stream, release the cuts."""
        self.reduce_bucket(self.nphases - 1)
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
        self._cuts = {k: [] for k in self._cuts}
        self._grads = {}
        self._nfwd = 0

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []
        for parent, idx in self._slots:
            parent.__dict__.get("_cut_fns", {}).pop(idx, None)
        self._slots = []
        if self._model is not None:
            self._model._dp_cut_fn = None
            self._model._dp_mark_fn = None
