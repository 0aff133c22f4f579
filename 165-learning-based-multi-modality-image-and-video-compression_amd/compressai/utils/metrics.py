"""Image-quality metrics of the evaluation scripts.

``psnr`` follows compressai/utils/eval_model/__main__t.py:89-91.  ``ms_ssim``
restates the multi-scale SSIM the reference imports from the third-party
``pytorch_msssim`` package (absent here; its published algorithm: 11-tap
Gaussian window, sigma 1.5, K = (0.01, 0.03), five scales with weights
(0.0448, 0.2856, 0.3001, 0.2363, 0.1333), 2x average pooling between
scales, ReLU on the contrast terms).  Evaluation-side torch ops, not on the
training hot path.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

_MS_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def psnr(a: torch.Tensor, b: torch.Tensor) -> float:
    mse = F.mse_loss(a.float(), b.float()).item()
    return -10 * math.log10(mse)


def _gauss_1d(size: int, sigma: float, device, dtype) -> torch.Tensor:
    coords = torch.arange(size, dtype=dtype, device=device) - size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    return (g / g.sum()).reshape(1, 1, 1, -1)


def _filter(x: torch.Tensor, win: torch.Tensor) -> torch.Tensor:
    """Separable 'valid' Gaussian filter per channel."""
    C = x.shape[1]
    out = F.conv2d(x, win.expand(C, 1, 1, -1), groups=C)
    return F.conv2d(out, win.transpose(2, 3).expand(C, 1, -1, 1), groups=C)


def _ssim(X, Y, win, data_range, K=(0.01, 0.03)):
    C1 = (K[0] * data_range) ** 2
    C2 = (K[1] * data_range) ** 2
    mu1, mu2 = _filter(X, win), _filter(Y, win)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = _filter(X * X, win) - mu1_sq
    sigma2_sq = _filter(Y * Y, win) - mu2_sq
    sigma12 = _filter(X * Y, win) - mu1_mu2
    cs_map = (2 * sigma12 + C2) / (sigma1_sq + sigma2_sq + C2)
    ssim_map = ((2 * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * cs_map
    return torch.flatten(ssim_map, 2).mean(-1), torch.flatten(cs_map, 2).mean(-1)


def ms_ssim(X: torch.Tensor, Y: torch.Tensor, data_range: float = 1.0, win_size: int = 11,
            win_sigma: float = 1.5) -> torch.Tensor:
    if X.shape != Y.shape or X.dim() != 4:
        raise ValueError(f"ms_ssim expects two [B, C, H, W] tensors of one shape, got {X.shape} / {Y.shape}")
    if min(X.shape[-2:]) <= (win_size - 1) * 2 ** 4:
        raise ValueError(f"image side must exceed {(win_size - 1) * 2 ** 4} for 5-scale MS-SSIM")
    X, Y = X.float(), Y.float()
    win = _gauss_1d(win_size, win_sigma, X.device, X.dtype)
    w = torch.tensor(_MS_WEIGHTS, device=X.device, dtype=X.dtype)
    mcs = []
    for i in range(len(_MS_WEIGHTS)):
        ssim_pc, cs = _ssim(X, Y, win, data_range)
        if i < len(_MS_WEIGHTS) - 1:
            mcs.append(torch.relu(cs))
            pad = [s % 2 for s in X.shape[2:]]
            X = F.avg_pool2d(X, kernel_size=2, padding=pad)
            Y = F.avg_pool2d(Y, kernel_size=2, padding=pad)
    vals = torch.stack(mcs + [torch.relu(ssim_pc)], dim=0)
    return torch.prod(vals ** w.view(-1, 1, 1), dim=0).mean()
