"""Per-parameter gradient error of the HIP path vs the CPU oracle (fp32 and float64) for one model config.

usage: python tools/grad_diff.py <zoo name> <width args comma-separated> <size> <batch> [--bf16] [--top N]
Prints every parameter whose HIP error exceeds 2e-3 (relative to the float64 tensor max) beside the fp32
oracle's own error, with the conv kernel each of the layer's launches used (compressai._ledger)."""
import argparse
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"),
          os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import cai_oracle as O  # noqa: E402


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    d = b.norm().item()
    return (a - b).norm().item() / (d if d > 0 else 1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("widths")
    ap.add_argument("size", type=int)
    ap.add_argument("batch", type=int)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("--no-kernels", action="store_true")
    a = ap.parse_args()
    from compressai import _ledger
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.zoo import model_architectures

    args = tuple(int(v) for v in a.widths.split(","))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    ref = O.ARCHS[a.name](*args)
    net = model_architectures[a.name](*args)
    net.load_state_dict(ref.state_dict())
    net = net.to(dev)
    x = torch.rand(a.batch, 3, a.size, a.size, generator=torch.Generator().manual_seed(a.seed))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(a.seed + 1))
    with feed:
        out_r = ref(x)
    O.RateDistortionLoss(6)(out_r, x)["loss"].backward()
    r64 = copy.deepcopy(ref).double()
    for p in r64.parameters():
        p.grad = None
    with O.NoiseFeed([n.double() for n in feed.drawn]):
        out64 = r64(x.double())
    O.RateDistortionLoss(6)(out64, x.double())["loss"].backward()
    q = [n.to(dev) for n in feed.drawn]
    set_noise_source(lambda t: q.pop(0))
    with _ledger.recording(keep_replay=False) as led:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.bf16):
            out = net(x.to(dev))
            c = RateDistortionLoss(6)(out, x.to(dev))
        c["loss"].backward()
        torch.cuda.synchronize()
    set_noise_source(None)
    print("x_hat", relerr(out["x_hat"], out64["x_hat"]), relerr(out_r["x_hat"], out64["x_hat"]))
    pr, p64 = dict(ref.named_parameters()), dict(r64.named_parameters())
    rows = []
    for n, p in net.named_parameters():
        if p64[n].grad is None:
            continue
        rows.append((relerr(p.grad, p64[n].grad), relerr(pr[n].grad, p64[n].grad), n, tuple(p.shape),
                     rel_l2(p.grad, p64[n].grad), rel_l2(pr[n].grad, p64[n].grad)))
    rows.sort(reverse=True)
    for e, e32, n, s, l2, l232 in rows[: a.top]:
        print(f"max {e:.3e} (cpu fp32 {e32:.3e})  l2 {l2:.3e} (cpu fp32 {l232:.3e})  {n} {s}")
    print("worst l2:", max(r[4] for r in rows), "cpu fp32 worst l2:", max(r[5] for r in rows))
    if a.no_kernels:
        return
    seen = {}
    for e in led.entries:
        if e.kind.startswith("conv"):
            seen.setdefault((e.kind, e.shape), e.kernel)
    for (k, s), kern in seen.items():
        print(f"{k:12s} {s:50s} {kern}")


if __name__ == "__main__":
    main()
