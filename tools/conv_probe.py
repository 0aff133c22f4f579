"""Standalone Conv2d / ConvTranspose2d fwd (+ optional backward) at one shape, for per-kernel PMC passes.
usage: python tools/conv_probe.py B Cin Cout H W k s transposed bwd reps"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "165-learning-based-multi-modality-image-and-video-compression_amd"))
import torch

from compressai.layers import Conv2d, ConvTranspose2d

B, ci, co, H, W, k, s, tr, bwd, reps = [int(v) for v in (sys.argv[1:11] if len(sys.argv) > 10
                                                        else [16, 128, 128, 128, 128, 5, 2, 0, 0, 20])]
m = (ConvTranspose2d(ci, co, k, stride=s, padding=k // 2, output_padding=s - 1) if tr
     else Conv2d(ci, co, k, stride=s, padding=k // 2)).cuda()
x = torch.randn(B, ci, H, W, device="cuda").requires_grad_(bool(bwd))
for _ in range(reps):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    if bwd:
        y.backward(torch.ones_like(y))
torch.cuda.synchronize()
print("ok", tuple(y.shape))
