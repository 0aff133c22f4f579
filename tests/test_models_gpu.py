"""Model-level parity on the GPU (exact-fp32 mode) against the CPU oracle.

Same state_dict, same inputs, same injected training noise.  Checked:
forward outputs, RD loss, every parameter gradient, one full optimizer step
(clip + Adam + aux), and eval-mode (entropy-estimation) bpp / PSNR within
1e-4 (north_star), with the round-to-index step bit-exact.
"""
import math

import pytest
import torch

import cai_oracle as O

pytestmark = pytest.mark.gpu

MODELS = ["bmshj2018-factorized", "bmshj2018-hyperprior", "mbt2018-mean", "mbt2018", "cheng2020-anchor",
          "cheng2020-attn"]


def _pair(name, N, M, dev):
    from compressai.zoo import model_architectures

    torch.manual_seed(0)
    args = (N,) if name.startswith("cheng2020") else (N, M)
    ref = O.ARCHS[name](*args)
    net = model_architectures[name](*args)
    net.load_state_dict(ref.state_dict())
    return ref, net.to(dev)


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


@pytest.mark.parametrize("name", MODELS)
def test_train_forward_backward_parity(cuda, name):
    _train_parity(cuda, name)


@pytest.mark.parametrize("stream", ["0", "1"])
@pytest.mark.parametrize("name", ["bmshj2018-hyperprior", "mbt2018-mean", "mbt2018", "cheng2020-anchor"])
def test_hyper_branch_stream_parity(cuda, monkeypatch, name, stream):
    """The hyper branch serial (0) and on its own stream (1), whatever the model's default (google.py)."""
    from compressai.models import google

    monkeypatch.setattr(google, "_HYPER_STREAM", stream)
    _train_parity(cuda, name)


def _train_parity(cuda, name):
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss

    ref, net = _pair(name, 32, 48, cuda)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(0))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(1))
    with feed:
        out_r = ref(x)
    cr = O.RateDistortionLoss(3)(out_r, x)
    cr["loss"].backward()
    q = [n.to(cuda) for n in feed.drawn]
    set_noise_source(lambda t: q.pop(0))
    try:
        out = net(x.to(cuda))
    finally:
        set_noise_source(None)
    assert not q
    c = RateDistortionLoss(3)(out, x.to(cuda))
    c["loss"].backward()
    assert relerr(out["x_hat"], out_r["x_hat"]) < 1e-4
    for k in out_r["likelihoods"]:
        assert relerr(out["likelihoods"][k], out_r["likelihoods"][k]) < 1e-4, k
    for k in ("loss", "bpp_loss", "mse_loss"):
        assert abs(c[k].item() - cr[k].item()) <= 1e-4 * max(1.0, abs(cr[k].item())), k
    pr = dict(ref.named_parameters())
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None:
            assert p.grad is None or p.grad.abs().max().item() == 0, n
            continue
        assert relerr(p.grad, gr) < 2e-3, n


@pytest.mark.parametrize("name", ["bmshj2018-hyperprior", "mbt2018-mean"])
def test_optimizer_step_parity(cuda, name):
    """train.py:155-186 step body: clip_grad_norm(1.0) + Adam + aux Adam, fp32."""
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.optim import configure_optimizers

    ref, net = _pair(name, 32, 48, cuda)
    opt_r, aux_r = O.configure_optimizers(ref, lr=1e-2, aux_lr=1e-1)
    opt, aux = configure_optimizers(net, lr=1e-2, aux_lr=1e-1)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(3))
    for it in range(2):
        feed = O.NoiseFeed(record=torch.Generator().manual_seed(10 + it))
        with feed:
            O.train_step(ref, O.RateDistortionLoss(1), x, opt_r, aux_r)
        q = [n.to(cuda) for n in feed.drawn]
        set_noise_source(lambda t: q.pop(0))
        try:
            opt.zero_grad()
            aux.zero_grad()
            out = net(x.to(cuda))
            RateDistortionLoss(1)(out, x.to(cuda))["loss"].backward()
            opt.step(max_norm=1.0)
            net.aux_loss().backward()
            aux.step()
        finally:
            set_noise_source(None)
    # Adam normalises each update to ~lr*sign(g) early on, so a gradient element
    # within rounding of zero can legitimately flip; require agreement for all
    # but a vanishing fraction of elements and a tight median.
    pr = dict(ref.named_parameters())
    diffs = torch.cat([(p.detach().cpu() - pr[n].detach()).abs().flatten() for n, p in net.named_parameters()])
    lr = 1e-2
    assert (diffs > 0.1 * lr).float().mean().item() < 1e-3
    assert diffs.median().item() < 1e-3 * lr


@pytest.mark.parametrize("zg", [False, True], ids=["keep-grads", "zero-grad-in-step"])
@pytest.mark.parametrize("large", [False, True], ids=["one-block", "two-launch"])
def test_fused_adam_matches_torch_adam(cuda, large, zg):
    """FusedAdam(+clip) == torch.optim.Adam + clip_grad_norm_ on identical gradients, on both launch paths of
    cai_adam_step (<= 65536 parameters: one block; above: norm partials + fused update), with and without
    the step consuming (zeroing) the gradients (zero_grad_in_step: zero_grad() then launches nothing and
    the next backward accumulates into the zeroed buffer)."""
    from compressai.optim import FusedAdam

    torch.manual_seed(9)
    shapes = [(128, 3, 5, 5), (128,), (7,), (64, 64)] + ([(192, 128, 3, 3)] if large else [])
    ref = [torch.nn.Parameter(torch.randn(s)) for s in shapes]
    dev = [torch.nn.Parameter(p.detach().clone().to(cuda)) for p in ref]
    opt_r = torch.optim.Adam(ref, lr=1e-3)
    opt = FusedAdam(dev, lr=1e-3, zero_grad_in_step=zg)
    for it in range(5):
        grads = [torch.randn(s) * (10.0 if it % 2 else 0.01) for s in shapes]
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        opt.zero_grad()
        for p, g in zip(dev, grads):
            p.grad.add_(g.to(cuda))          # accumulate, as a backward does
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt_r.step()
        opt.step(max_norm=1.0)
        if zg:
            assert float(opt.flat_grad.abs().max()) == 0.0
    for a, b in zip(dev, ref):
        assert (a.detach().cpu() - b.detach()).abs().max().item() < 1e-6


@pytest.mark.parametrize("name", MODELS)
def test_entropy_estimation_eval_parity(cuda, name):
    """utils/eval_model/__main__t.py:149-211: eval-mode bpp / PSNR within 1e-4."""
    from compressai.losses import RateDistortionLoss

    ref, net = _pair(name, 64, 96, cuda)
    ref.eval()
    net.eval()
    x = torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(5))
    r = O.entropy_estimation(ref, x)
    with torch.no_grad():
        out = net(x.to(cuda))
    npix = x.shape[2] * x.shape[3]
    bpp = sum(torch.log(l.float()).sum().item() for l in out["likelihoods"].values()) / (-math.log(2) * npix)
    mse = torch.mean((out["x_hat"].cpu() - x) ** 2).item()   # unclamped, as __main__t.py:169,207
    psnr = -10 * math.log10(mse)
    assert abs(bpp - r["bpp"]) <= 1e-4 * max(1.0, r["bpp"]), (bpp, r["bpp"])
    assert abs(psnr - r["psnr"]) <= 1e-4 * r["psnr"], (psnr, r["psnr"])


def test_bf16_training_step_is_close(cuda):
    """autocast (bf16) path: loss within 2% of the fp32 oracle on the same step."""
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss

    ref, net = _pair("bmshj2018-hyperprior", 128, 192, cuda)
    x = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(7))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(8))
    with feed:
        cr = O.RateDistortionLoss(1)(ref(x), x)
    q = [n.to(cuda) for n in feed.drawn]
    set_noise_source(lambda t: q.pop(0))
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = net(x.to(cuda))
            c = RateDistortionLoss(1)(out, x.to(cuda))
    finally:
        set_noise_source(None)
    c["loss"].backward()
    assert abs(c["loss"].item() - cr["loss"].item()) < 0.02 * abs(cr["loss"].item())
    assert all(torch.isfinite(p.grad).all() for p in net.parameters() if p.grad is not None)
