"""Layer zoo (reference: compressai/layers/layers.py:40-296).

MaskedConv2d follows layers.py:52-78: the weight is masked in place before
every call (so gradients reach masked taps exactly as in the reference), then
the conv runs on the HIP implicit-GEMM kernel.
"""
from typing import Any

import torch
import torch.nn as nn

from .conv import Conv2d, ConvTranspose2d

__all__ = ["MaskedConv2d", "conv1x1", "conv3x3"]


class MaskedConv2d(Conv2d):
    def __init__(self, *args: Any, mask_type: str = "A", **kwargs: Any):
        super().__init__(*args, **kwargs)
        if mask_type not in ("A", "B"):
            raise ValueError(f'Invalid "mask_type" value "{mask_type}"')
        self.register_buffer("mask", torch.ones_like(self.weight.data))
        _, _, h, w = self.mask.size()
        self.mask[:, :, h // 2, w // 2 + (mask_type == "B"):] = 0
        self.mask[:, :, h // 2 + 1:] = 0

    def run(self, x, **kw):
        self.weight.data *= self.mask
        return super().run(x, **kw)


def conv3x3(in_ch: int, out_ch: int, stride: int = 1) -> nn.Module:
    return Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def conv1x1(in_ch: int, out_ch: int, stride: int = 1) -> nn.Module:
    return Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)
