"""ste_round (reference: compressai/ops/ops.py:35-49): round with identity gradient."""
import torch


def ste_round(x: torch.Tensor) -> torch.Tensor:
    return torch.round(x) - x.detach() + x
