"""Data parallelism: one process per GPU, gradient all-reduce over RCCL/xGMI.

The reference trains with single-process nn.DataParallel
(examples/train.py:101-108,413); here each rank owns a GPU, processes its own
patches, and the only exchange per step is ONE all-reduce (average) of the
flat gradient buffer of FusedAdam (20.3 MB fp32 for bmshj2018-hyperprior).
The aux loss (EntropyBottleneck.loss) depends only on replicated parameters,
so its gradients are identical on every rank and need no exchange.
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
