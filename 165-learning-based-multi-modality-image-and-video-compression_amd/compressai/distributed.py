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


class OverlappedAllReduce:
    """Two-bucket gradient all-reduce overlapped with the backward of the model's tail.

    The backward runs in two phases: ``backward_head(loss)`` differentiates down to the cut tensors and
    into every other parameter (``torch.autograd.backward(loss, inputs=[*cut, *head_params])``), so
    flat_grad[:split] -- every gradient but the tail's (FusedAdam layout from
    configure_optimizers(..., tail=model.dp_tail)) -- is final; ``reduce_head()`` all-reduces it on a side
    stream while ``backward_tail()`` runs the tail's backward on the compute stream; ``finish()``
    all-reduces flat_grad[split:] and joins the streams.  Each phase can be captured in its own HIP
    graph; the collectives stay outside the graphs (stream order only, no events).

    `tail`: a model with a ``_dp_cut`` marker (CompressionModel: the cut the model itself declares), or any
    module whose output is a cut (a forward hook marks it: e.g. ``net.g_a`` of the zoo models).

    Memory: backward_head keeps the graph (retain_graph) because backward_tail still needs the tail's saved
    tensors; the head's saved tensors are released when the caller drops its loss tensor (bench.py's step
    drops it on return) -- the serial backward's peak otherwise."""

    def __init__(self, flat_grad: torch.Tensor, split: int, tail: torch.nn.Module, head_params):
        self.head = flat_grad[:split]
        self.tail = flat_grad[split:]
        self.head_params = [p for p in head_params if p.requires_grad]
        self.side = torch.cuda.Stream(device=flat_grad.device)
        self._ys = []
        self._model = None
        self._handles = []
        if hasattr(tail, "_dp_cut") and hasattr(tail, "dp_tail"):
            self._model = tail
            tail._dp_cut_fn = self._mark
        else:
            self._handles.append(tail.register_forward_hook(self._keep))
        # each forward starts a new set of cut tensors: one that never reached backward_tail (a validation
        # pass, a plain backward) neither leaks into the next step nor keeps its cut tensors alive
        self._handles.append(tail.register_forward_pre_hook(self._reset))

    @classmethod
    def for_model(cls, model: torch.nn.Module, opt):
        """The exchange of `model` over FusedAdam `opt` built by configure_optimizers(model, tail=model.dp_tail)."""
        tail = tuple(model.dp_tail)
        head = [p for n, p in model.named_parameters()
                if not n.startswith(tail) and not n.endswith(".quantiles")]
        return cls(opt.flat_grad, opt.tail_offset, model, head)

    def _reset(self, module, inputs):
        self._ys = []

    def _mark(self, *ts):
        # only a forward that can be differentiated marks its cut (no_grad / eval passes go through as is)
        if not torch.is_grad_enabled() or not any(t.requires_grad for t in ts):
            return ts
        # boundary nodes: phase 1's capture of a cut tensor's gradient may execute its grad_fn, which for
        # the product convs writes parameter gradients as a side effect; an identity node in between has none
        out = tuple(_Boundary.apply(t) for t in ts)
        self._ys.extend(out)
        return out

    def _keep(self, module, inputs, output):
        return self._mark(output)[0]

    def backward_head(self, loss: torch.Tensor):
        if not self._ys:
            raise RuntimeError("OverlappedAllReduce: the forward did not reach the cut")
        # retain_graph: the engine releases the saved tensors of every node of the graph it was given,
        # including the tail's, which backward_tail still needs
        from ._ops import loss_seed

        torch.autograd.backward(loss, grad_tensors=loss_seed(loss), inputs=list(self._ys) + self.head_params,
                                retain_graph=True)

    def backward_tail(self):
        ys, self._ys = self._ys, []
        used = [y for y in ys if y.grad is not None]
        torch.autograd.backward(used, grad_tensors=[y.grad for y in used])

    def reduce_head(self):
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            if self.head.numel():
                allreduce_mean_(self.head)

    def finish(self):
        """All-reduce the tail bucket after the whole backward, then join the side stream."""
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            if self.tail.numel():
                allreduce_mean_(self.tail)
        cur.wait_stream(self.side)

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []
        if self._model is not None:
            self._model._dp_cut_fn = None
