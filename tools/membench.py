"""HBM calibration beside the GDN kernels: torch copy / fill / read of a B16 x 128 x 128 x 128 bf16 tensor
(the hyperprior's largest GDN activation) and the product GDN forward / backward on it, HIP-event timed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))
import torch  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


dev = torch.device("cuda")
x = torch.randn(16, 128, 128, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.empty_like(x)
nb = x.numel() * 2
us = timeit(lambda: y.copy_(x))
print(f"copy  {us:7.1f} us  {2 * nb / us / 1e6:6.2f} TB/s (read+write {2 * nb / 1e6:.0f} MB)")
us = timeit(lambda: y.fill_(1.0))
print(f"fill  {us:7.1f} us  {nb / us / 1e6:6.2f} TB/s")
us = timeit(lambda: x.sum(dtype=torch.float32))
print(f"sum   {us:7.1f} us  {nb / us / 1e6:6.2f} TB/s")
from compressai.layers import GDN  # noqa: E402

for inv in (False, True):
    g = GDN(128, inverse=inv).to(dev)
    xr = x.detach().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = g(xr)
    gy = torch.randn_like(out)

    def fw():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            g(x)
    us = timeit(fw)
    print(f"gdn fwd inv={inv} (incl. python) {us:7.1f} us  {2 * nb / us / 1e6:6.2f} TB/s")

    def fb():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            o = g(xr)
        o.backward(gy)
    us = timeit(fb, 20)
    print(f"gdn fwd+bwd inv={inv} {us:7.1f} us")
