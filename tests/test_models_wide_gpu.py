"""Model-level parity at the configured widths of every BASELINE config (SURVEY.md §8 preamble,
zoo/image.py:190-245): fp32 mode against the CPU oracle (outputs, likelihoods, RD loss, every parameter
gradient), and the bf16 autocast mode bounded on x_hat, likelihoods and gradients -- not only the loss.

fp32 bars are the north_star's (1e-4 on outputs / likelihoods / loss; 2e-3 on gradients, relative to the
tensor's max), measured against a float64 run of the oracle; where fp32 arithmetic itself cannot meet them (the
CPU fp32 oracle misses a cheng2020-attn attention-branch gradient by 6.7e-3 against float64), the HIP path
must stay within 2x the CPU fp32 error.  bf16 bars are written per quantity below; they are the measured bf16 errors on MI355X with
about 3x headroom (bf16 keeps 8 mantissa bits, so a single rounding is 2^-9 = 2e-3 relative, and the
errors of ~10-20 stacked layers add up).
"""
import math

import pytest
import torch

import cai_oracle as O

pytestmark = pytest.mark.gpu

# (zoo name, constructor widths, patch size): the quality -> (N, M) table of zoo/image.py:190-245
WIDE = [
    ("bmshj2018-factorized", (192, 320), 64),     # C1 at q6-8
    ("bmshj2018-hyperprior", (128, 192), 128),    # C2 (q1-5)
    ("bmshj2018-hyperprior", (192, 320), 128),    # C2' (q6-8)
    ("mbt2018-mean", (128, 192), 128),            # C3 (q1-4)
    ("mbt2018-mean", (192, 320), 128),            # C3 (q5-8)
    ("mbt2018", (192, 192), 64),                  # C3' (+context, q1-4)
    ("cheng2020-anchor", (192,), 64),             # cheng2020 q4-6
    ("cheng2020-attn", (192,), 64),               # C4 (q6)
]


def _ids(c):
    return f"{c[0]}-{'x'.join(map(str, c[1]))}-{c[2]}"


def _pair(name, args, dev):
    from compressai.zoo import model_architectures

    torch.manual_seed(0)
    ref = O.ARCHS[name](*args)
    net = model_architectures[name](*args)
    net.load_state_dict(ref.state_dict())
    return ref, net.to(dev)


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def _run_both(name, args, size, cuda, bf16, seed=0, batch=2, keep=False):
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss

    ref, net = _pair(name, args, cuda)
    x = torch.rand(batch, 3, size, size, generator=torch.Generator().manual_seed(seed))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(seed + 1))
    with feed:
        out_r = ref(x)
    cr = O.RateDistortionLoss(1)(out_r, x)
    cr["loss"].backward()
    q = [n.to(cuda) for n in feed.drawn]
    set_noise_source(lambda t: q.pop(0))
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            out = net(x.to(cuda))
            c = RateDistortionLoss(1)(out, x.to(cuda))
    finally:
        set_noise_source(None)
    assert not q
    c["loss"].backward()
    if keep:
        return ref, net, out_r, out, cr, c, feed.drawn, x
    return ref, net, out_r, out, cr, c


def _oracle64(ref, x, noises):
    """The oracle in float64 on the same weights and noise: the truth both fp32 paths are measured against."""
    import copy

    r64 = copy.deepcopy(ref).double()
    for p in r64.parameters():
        p.grad = None
    with O.NoiseFeed([n.double() for n in noises]):
        out = r64(x.double())
    cr = O.RateDistortionLoss(1)(out, x.double())
    cr["loss"].backward()
    return r64, out, cr


@pytest.mark.parametrize("case", WIDE, ids=_ids)
def test_fp32_parity_at_configured_width(cuda, case):
    """fp32 HIP path vs the fp32 CPU oracle, both measured against the float64 oracle: the HIP error must be
    within the north_star bar (1e-4 outputs, 2e-3 gradients) or, where fp32 itself cannot hold that bar (a
    gradient summed from cancelling terms), within 2x the fp32 CPU oracle's own error."""
    name, args, size = case
    ref, net, out_r, out, cr, c, drawn, x = _run_both(name, args, size, cuda, bf16=False, keep=True)
    r64, out64, cr64 = _oracle64(ref, x, drawn)

    def check(a, a32, a64, bar, what):
        e, e32 = relerr(a, a64), relerr(a32, a64)
        assert e < max(bar, 2 * e32), (what, e, e32)

    check(out["x_hat"], out_r["x_hat"], out64["x_hat"], 1e-4, "x_hat")
    for k in out_r["likelihoods"]:
        check(out["likelihoods"][k], out_r["likelihoods"][k], out64["likelihoods"][k], 1e-4, k)
    for k in ("loss", "bpp_loss", "mse_loss"):
        assert abs(c[k].item() - cr[k].item()) <= 1e-4 * max(1.0, abs(cr[k].item())), k
    pr, p64 = dict(ref.named_parameters()), dict(r64.named_parameters())
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None:
            assert p.grad is None or p.grad.abs().max().item() == 0, n
            continue
        check(p.grad, gr, p64[n].grad, 2e-3, n)


# bf16 bars: x_hat and likelihoods relative to the tensor's max; the whole gradient vector's cosine against the
# oracle's (`GRAD_COS`); per parameter tensor its cosine (`TENSOR_COS`).  The per-tensor max error relative to the
# tensor's max is printed, not bounded: for tensors dominated by a few large entries it reads 0.2-0.7 while
# the tensor's cosine stays >= 0.995.  Measured on MI355X (hyperprior 192x320): x_hat 2.4e-3, lik 4.5e-3, loss 3e-5, cosine 0.999999;
# the lowest per-tensor cosine over five configs is 0.9951 (h_s / h_a, whose gradients arrive through the
# GaussianConditional scale input).
BF16_XHAT = 1e-2
BF16_LIK = 2e-2
BF16_LOSS = 1e-3
GRAD_COS = 0.9999
TENSOR_COS = 0.98

BF16 = [
    ("bmshj2018-hyperprior", (128, 192), 128),
    ("bmshj2018-hyperprior", (192, 320), 128),
    ("mbt2018-mean", (128, 192), 128),
    ("mbt2018", (192, 192), 64),
    ("cheng2020-attn", (192,), 64),
]


@pytest.mark.parametrize("case", BF16, ids=_ids)
def test_bf16_bounds_at_configured_width(cuda, case):
    name, args, size = case
    ref, net, out_r, out, cr, c = _run_both(name, args, size, cuda, bf16=True, seed=4)
    ex = relerr(out["x_hat"], out_r["x_hat"])
    el = {k: relerr(out["likelihoods"][k], out_r["likelihoods"][k]) for k in out_r["likelihoods"]}
    eloss = abs(c["loss"].item() - cr["loss"].item()) / abs(cr["loss"].item())
    pr = dict(ref.named_parameters())
    worst, tcos, dots, na, nb = {}, {}, 0.0, 0.0, 0.0
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None or p.grad is None:
            continue
        g = p.grad.detach().float().cpu()
        assert torch.isfinite(g).all(), n
        worst[n] = relerr(g, gr)
        tcos[n] = float(torch.nn.functional.cosine_similarity(g.double().flatten(), gr.double().flatten(), dim=0))
        dots += float((g.double() * gr.double()).sum())
        na += float((g.double() ** 2).sum())
        nb += float((gr.double() ** 2).sum())
    cos = dots / math.sqrt(na * nb)
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:3]
    low = sorted(tcos.items(), key=lambda kv: kv[1])[:3]
    print(f"\nbf16 {_ids(case)}: x_hat {ex:.3e} lik {el} loss {eloss:.3e} grad cos {cos:.6f} worst {top} "
          f"lowest tensor cos {low}")
    assert ex < BF16_XHAT
    for k, v in el.items():
        assert v < BF16_LIK, k
    assert eloss < BF16_LOSS
    assert cos > GRAD_COS
    assert low[0][1] > TENSOR_COS, low


@pytest.mark.parametrize("name,args", [("cheng2020-attn", (192,)), ("bmshj2018-hyperprior", (192, 320)),
                                       ("mbt2018", (192, 192))])
def test_eval_parity_at_configured_width(cuda, name, args):
    """utils/eval_model/__main__t.py:149-211 (entropy estimation, unclamped PSNR) at q6 widths, 1e-4."""
    ref, net = _pair(name, args, cuda)
    ref.eval()
    net.eval()
    x = torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(5))
    r = O.entropy_estimation(ref, x)
    with torch.no_grad():
        out = net(x.to(cuda))
    npix = x.shape[2] * x.shape[3]
    bpp = sum(torch.log(l.float()).sum().item() for l in out["likelihoods"].values()) / (-math.log(2) * npix)
    mse = torch.mean((out["x_hat"].cpu() - x) ** 2).item()
    psnr = -10 * math.log10(mse)
    assert abs(bpp - r["bpp"]) <= 1e-4 * max(1.0, r["bpp"]), (bpp, r["bpp"])
    assert abs(psnr - r["psnr"]) <= 1e-4 * r["psnr"], (psnr, r["psnr"])
