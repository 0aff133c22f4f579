"""Standalone GDN / IGDN backward at one size, for per-kernel PMC passes (tools/pmc_kernels.sh style).
usage: python tools/gdn_probe.py [B H W C inverse reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "165-learning-based-multi-modality-image-and-video-compression_amd"))
import torch

from compressai.layers import GDN

B, H, W, C, inv, reps = [int(v) for v in (sys.argv[1:7] if len(sys.argv) > 6 else [16, 128, 128, 128, 0, 20])]
m = GDN(C, inverse=bool(inv)).cuda()
x = torch.randn(B, C, H, W, device="cuda").requires_grad_()
g = torch.randn(B, C, H, W, device="cuda")
with torch.autocast("cuda", dtype=torch.bfloat16):
    y = m(x)
for _ in range(reps):
    (gx,) = torch.autograd.grad(y, x, g, retain_graph=True)
torch.cuda.synchronize()
print("ok", gx.shape)
