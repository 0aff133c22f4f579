"""GPU diagnostic: the two-phase backward of compressai.distributed.OverlappedAllReduce (head inputs, then g_a)
against one ordinary backward on the product ScaleHyperprior, fp32 and bf16."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))
import torch  # noqa: E402

from compressai.entropy_models import set_noise_source  # noqa: E402
from compressai.losses import RateDistortionLoss  # noqa: E402
from compressai.models import ScaleHyperprior  # noqa: E402
from compressai.optim import configure_optimizers  # noqa: E402
from compressai.distributed import OverlappedAllReduce  # noqa: E402

dev = torch.device("cuda:0")
for bf16 in (False, True):
    for tail in ((), ("g_a.",)):
        torch.manual_seed(0)
        net = ScaleHyperprior(32, 48).to(dev).train()
        opt, aux = configure_optimizers(net, tail=tail)
        x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1)).to(dev)
        noise = [torch.zeros(2, 32, 1, 1, device=dev), torch.zeros(2, 48, 4, 4, device=dev)]
        res = {}
        for mode in ("plain", "two"):
            q = list(noise)
            set_noise_source(lambda t: q.pop(0))
            opt.zero_grad()
            head = [p for n, p in net.named_parameters() if not n.startswith("g_a.") and not n.endswith(".quantiles")]
            sync = OverlappedAllReduce(opt.flat_grad, opt.tail_offset, net.g_a, head) if mode == "two" else None
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(x)
                loss = RateDistortionLoss(1)(out, x)["loss"]
            if sync:
                sync.backward_head(loss)
                sync.backward_tail()
                sync.remove()
            else:
                loss.backward()
            set_noise_source(None)
            torch.cuda.synchronize()
            res[mode] = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
        bad = []
        for n, g in res["plain"].items():
            e = (res["two"][n] - g).abs().max().item() / max(g.abs().max().item(), 1e-30)
            if e > 1e-6:
                bad.append((n, e))
        print(f"bf16={bf16} tail={tail}: {len(bad)} mismatching params {bad[:6]}")
