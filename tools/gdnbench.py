"""GDN forward / backward on the hyperprior's largest layer (16 x 128 x 128 x 128 bf16), 30 launches each, for
rocprofv3 counter passes (tools/pmc_gdn.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))
import torch  # noqa: E402

from compressai.layers import GDN  # noqa: E402

dev = torch.device("cuda")
x = torch.randn(16, 128, 128, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
g = GDN(128).to(dev)
xr = x.detach().requires_grad_(True)
with torch.autocast("cuda", dtype=torch.bfloat16):
    out = g(xr)
gy = torch.randn_like(out)
for _ in range(30):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        o = g(xr)
    o.backward(gy)
torch.cuda.synchronize()
print("ok")
