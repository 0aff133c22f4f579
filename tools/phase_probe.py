"""Timing probe: repeated g_s[4] forwards (ConvTranspose2d 128->128 k5 s2, 64^2 -> 128^2, B=16, bf16) on the
halo-staged phase kernel; results are not checked (probe builds compute garbage on purpose)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))
import torch  # noqa: E402

from compressai.layers import ConvTranspose2d  # noqa: E402

dec = ConvTranspose2d(128, 128, 5, stride=2, padding=2, output_padding=1).cuda()
x = torch.randn(16, 128, 64, 64, device="cuda")
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
    for _ in range(30):
        dec(x)
torch.cuda.synchronize()
print("ok")
