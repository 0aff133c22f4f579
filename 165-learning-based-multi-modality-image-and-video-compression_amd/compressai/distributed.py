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
    """Where the cut at the input of child `name` ("g_a.4") is marked: the parent's cut slot for a product
    Sequential (compressai.layers.Sequential), else the child's forward pre-hook."""
    from .layers.conv import Sequential

    parent, idx = name.rsplit(".", 1)
    pm = model.get_submodule(parent)
    if isinstance(pm, Sequential):
        return (pm, int(idx))
    return model.get_submodule(name)


class OverlappedAllReduce:
    """Bucketed gradient all-reduce overlapped with the backward.

    The flat gradient buffer of FusedAdam (configure_optimizers(..., tail=model.dp_tail,
    tail_cuts=model.dp_tail_cuts)) holds the buckets in the order the backward finishes them: the head
    (everything but the tail), then the tail's pieces from the loss side down to the input.  The backward
    runs in one phase per bucket: ``backward_head(loss)`` differentiates down to the model's cut
    (``torch.autograd.backward(loss, inputs=[*cut, *head_params])``), so bucket 0 is final;
    ``backward_phase(i)`` continues from cut i-1 down to cut i (the input of the tail child named by
    dp_tail_cuts[i-1]) or, for the last one, to the input.  ``reduce_bucket(i)`` all-reduces bucket i on a
    side stream while the next phase runs on the compute stream; ``finish()`` all-reduces the last bucket and
    joins the streams.  Each phase can be captured in its own HIP graph; the collectives stay outside the
    graphs (stream order only, no events).  ``reduce_head()`` / ``backward_tail()`` are the eager two-call
    form (every tail phase, each bucket all-reduced once the phase after it is queued).

    `tail`: a model with a ``_dp_cut`` marker (CompressionModel: the cut the model itself declares), or any
    module whose output is a cut (a forward hook marks it: e.g. ``net.g_a`` of the zoo models).

    Cut tensors accumulate over the grad-enabled forwards of a step (micro-batches summed into one loss) and
    are released by ``finish()``; a plain ``loss.backward()`` outside the phases (no exchange) releases the
    ones it differentiated through, so they never leak into the next step.  The cuts of a grad-enabled
    forward the step's loss does not depend on (one computed for logging, never backpropagated) are dropped
    by ``backward_head`` (a reachability walk from the loss, only when more than one forward marked a cut).
    Cut lists must come in backward order (``optim.check_tail_cuts``).

    Memory: each phase keeps the graph (retain_graph) because the later phases still need the tail's saved
    tensors; they are released when the caller drops its loss tensor (bench.py's step drops it on return) --
    the serial backward's peak otherwise."""

    def __init__(self, flat_grad: torch.Tensor, split, tail: torch.nn.Module, head_params,
                 cut_modules=(), stage_params=None):
        bounds = list(split) if isinstance(split, (list, tuple)) else [0, int(split), flat_grad.numel()]
        if len(bounds) != len(cut_modules) + 3 and not (len(bounds) == 2 and not cut_modules):
            raise ValueError("OverlappedAllReduce: one bucket per cut piece expected "
                             f"({len(cut_modules) + 2} buckets for {len(cut_modules)} tail cuts, bounds {bounds})")
        self.buckets = [flat_grad[bounds[i]:bounds[i + 1]] for i in range(len(bounds) - 1)]
        self.head, self.tail = self.buckets[0], flat_grad[bounds[1]:] if len(bounds) > 2 else flat_grad[:0]
        self.head_params = [p for p in head_params if p.requires_grad]
        self.stage_params = [[p for p in ps if p.requires_grad] for ps in (stage_params or [])]
        # (a CPU buffer -- the gloo tests of the phase logic -- reduces synchronously, no side stream)
        self.side = torch.cuda.Stream(device=flat_grad.device) if flat_grad.is_cuda else None
        self._cuts = [[] for _ in range(max(1, len(self.buckets) - 1))]   # cut tensors of each tail phase
        self._in_phase = False
        self._nfwd = 0                  # grad-enabled forwards that marked cut 0 since the last step
        self._model = None
        self._handles = []
        self._slots = []
        if hasattr(tail, "_dp_cut") and hasattr(tail, "dp_tail"):
            self._model = tail
            tail._dp_cut_fn = lambda *ts: self._mark(0, *ts)
        else:
            self._handles.append(tail.register_forward_hook(lambda m, i, o: self._mark(0, o)[0]))
        for k, m in enumerate(cut_modules):
            if isinstance(m, tuple):
                # (parent Sequential, child index): the product Sequential runs its children through .run()
                # (conv + activation epilogue fusion), so the cut goes into its own cut slots
                parent, idx = m
                slots = parent.__dict__.setdefault("_cut_fns", {})
                slots[idx] = lambda x, k=k: self._mark(k + 1, x)
                self._slots.append((parent, idx))
            else:
                self._handles.append(m.register_forward_pre_hook(
                    lambda mod, inputs, k=k: (self._mark(k + 1, inputs[0]),) + tuple(inputs[1:])))

    @classmethod
    def for_model(cls, model: torch.nn.Module, opt):
        """The exchange of `model` over FusedAdam `opt` built by configure_optimizers(model,
        tail=model.dp_tail, tail_cuts=model.dp_tail_cuts); a buffer built without the cuts gets two buckets."""
        from .optim import check_tail_cuts, dp_stage

        tail = tuple(model.dp_tail)
        bounds = list(getattr(opt, "bucket_bounds", [0, opt.tail_offset, opt.numel]))
        cuts = check_tail_cuts(getattr(model, "dp_tail_cuts", ())) if len(bounds) > 3 else ()
        main = [(n, p) for n, p in model.named_parameters() if not n.endswith(".quantiles")]
        head = [p for n, p in main if dp_stage(n, tail, cuts) == 0]
        stages = [[p for n, p in main if dp_stage(n, tail, cuts) == s] for s in range(1, len(cuts) + 2)]
        return cls(opt.flat_grad, bounds, model, head, [_cut_site(model, c) for c in cuts], stages)

    @property
    def nphases(self) -> int:
        return len(self.buckets)

    def _mark(self, k, *ts):
        # only a forward that can be differentiated marks its cut (no_grad / eval passes go through as is)
        if not torch.is_grad_enabled() or not any(t.requires_grad for t in ts):
            return ts[0] if k else ts
        # boundary nodes: a phase's capture of a cut tensor's gradient may execute its grad_fn, which for
        # the product convs writes parameter gradients as a side effect; an identity node in between has none
        out = tuple(_Boundary.apply(t) for t in ts)
        if k == 0:
            self._nfwd += 1
        for t in out:
            # a backward outside the phases (a plain loss.backward()) releases the cut (by id: a reference in the
            # hook would keep the tensor, and with it its graph, alive until the cycle collector runs)
            t.register_hook(lambda g, tid=id(t), k=k: self._release(k, tid))
        self._cuts[k].extend(out)
        return out[0] if k else out

    def _release(self, k, tid):
        if not self._in_phase:
            self._cuts[k] = [c for c in self._cuts[k] if id(c) != tid]
            if k == 0 and not self._cuts[0]:
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
        self._cuts = [[t for t in c if t.grad_fn in seen] for c in self._cuts]
        self._nfwd = 1

    def _backward(self, roots, grads, inputs):
        self._in_phase = True
        try:
            torch.autograd.backward(roots, grad_tensors=grads, inputs=inputs or None, retain_graph=bool(inputs))
        finally:
            self._in_phase = False

    def backward_head(self, loss: torch.Tensor):
        self._prune(loss)
        if not self._cuts[0]:
            raise RuntimeError("OverlappedAllReduce: the forward did not reach the cut")
        from ._ops import loss_seed

        # retain_graph: the engine releases the saved tensors of every node of the graph it was given,
        # including the tail's, which the later phases still need
        self._backward(loss, loss_seed(loss), list(self._cuts[0]) + self.head_params)

    def backward_phase(self, i: int):
        """Tail phase i (1 .. nphases - 1): from cut i - 1's gradients down to cut i (all of it for the last)."""
        ys = [y for y in self._cuts[i - 1] if y.grad is not None]
        last = i == self.nphases - 1
        inputs = [] if last else list(self._cuts[i]) + self.stage_params[i - 1]
        if ys:
            self._backward(ys, [y.grad for y in ys], inputs)

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
        """Every tail phase, eagerly: bucket i is all-reduced while phase i + 1 runs (the last by finish())."""
        for i in range(1, self.nphases):
            self.backward_phase(i)
            if i < self.nphases - 1:
                self.reduce_bucket(i)

    def finish(self):
        """All-reduce the last bucket after the whole backward, join the side stream, release the cuts."""
        self.reduce_bucket(self.nphases - 1)
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
        self._cuts = [[] for _ in self._cuts]
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
