"""Data parallelism: one process per GPU, gradient all-reduce over RCCL/xGMI.

The reference trains with single-process nn.DataParallel
(examples/train.py:101-108,413); here each rank owns a GPU, processes its own
patches, and the only exchange per step is the all-reduce (average) of the
flat gradient buffer of FusedAdam (20.3 MB fp32 for bmshj2018-hyperprior).
The aux loss (EntropyBottleneck.loss) depends only on replicated parameters,
so its gradients are identical on every rank and need no exchange.

OverlappedAllReduce splits that exchange in two buckets: every gradient but
the analysis transform's is final once the backward has reached g_a's output
y (y feeds every other branch), so that bucket is all-reduced on a side
stream while g_a's backward runs; the g_a bucket follows.
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
    """Two-bucket gradient all-reduce overlapped with the backward of `tail_module`.

    The backward runs in two phases: ``backward_head(loss)`` differentiates down to tail_module's output y
    and into every other parameter (``torch.autograd.backward(loss, inputs=[y, *head_params])``), so
    flat_grad[:split] -- every gradient but tail_module's (FusedAdam layout from
    configure_optimizers(..., tail=("g_a.",))) -- is final; ``reduce_head()`` all-reduces it on a side
    stream while ``backward_tail()`` runs tail_module's backward on the compute stream; ``finish()``
    all-reduces flat_grad[split:] and joins the streams.  Each phase can be captured in its own HIP
    graph; the collectives stay outside the graphs (stream order only, no events)."""

    def __init__(self, flat_grad: torch.Tensor, split: int, tail_module: torch.nn.Module, head_params):
        self.head = flat_grad[:split]
        self.tail = flat_grad[split:]
        self.head_params = [p for p in head_params if p.requires_grad]
        self.side = torch.cuda.Stream(device=flat_grad.device)
        self._y = None
        self._handle = tail_module.register_forward_hook(self._keep)

    def _keep(self, module, inputs, output):
        # the boundary node: phase 1's capture of y's gradient may execute y's grad_fn, which for the
        # product convs writes parameter gradients as a side effect; an identity node in between has none
        self._y = _Boundary.apply(output)
        return self._y

    def backward_head(self, loss: torch.Tensor):
        if self._y is None:
            raise RuntimeError("OverlappedAllReduce: the tail module did not run in this forward")
        # retain_graph: the engine releases the saved tensors of every node of the graph it was given,
        # including g_a's, which backward_tail still needs
        torch.autograd.backward(loss, inputs=[self._y] + self.head_params, retain_graph=True)

    def backward_tail(self):
        y, self._y = self._y, None
        torch.autograd.backward(y, grad_tensors=y.grad)

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
        self._handle.remove()
