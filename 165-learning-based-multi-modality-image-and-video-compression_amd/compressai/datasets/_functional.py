"""The few torchvision transforms the reference's loaders use, restated on PIL + torch (torchvision is not
part of this stack).  Each keeps torchvision's semantics for 8-bit images:

* ``to_tensor``: ``transforms.ToTensor`` -- HWC uint8 -> CHW float in [0, 1] (1 channel for mode "L");
* ``resize``: ``transforms.Resize`` on a tensor -- bilinear, ``align_corners=False``, antialiased;
* ``hflip``: ``transforms.functional.hflip`` -- mirror the last axis;
* ``center_crop``: ``transforms.CenterCrop`` -- top / left offsets ``round((H - h) / 2)``, zero padding when
  the image is smaller than the crop.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F


def to_tensor(img) -> torch.Tensor:
    arr = np.array(img)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    t = torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1)))
    if arr.dtype == np.uint8:
        return t.float().div_(255)
    return t.float()


def resize(x: torch.Tensor, size: Sequence[int]) -> torch.Tensor:
    h, w = int(size[0]), int(size[1])
    if tuple(x.shape[-2:]) == (h, w):
        return x
    return F.interpolate(x.unsqueeze(0), size=(h, w), mode="bilinear", align_corners=False,
                         antialias=True).squeeze(0)


def hflip(x: torch.Tensor) -> torch.Tensor:
    return x.flip(-1)


def center_crop(x: torch.Tensor, size: Tuple[int, int]) -> torch.Tensor:
    ch, cw = size
    h, w = x.shape[-2:]
    if ch > h or cw > w:
        pt, pl = max(ch - h, 0) // 2, max(cw - w, 0) // 2
        x = F.pad(x, (pl, max(cw - w, 0) - pl, pt, max(ch - h, 0) - pt))
        h, w = x.shape[-2:]
    top, left = int(round((h - ch) / 2.0)), int(round((w - cw) / 2.0))
    return x[..., top:top + ch, left:left + cw]
