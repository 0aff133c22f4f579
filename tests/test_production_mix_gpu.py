"""Model-level checks at the BASELINE configs' own sizes, so the kernels the bench runs are the kernels
under test (the 192-channel conv tiles are gated on grid size: conv_halo_s1_kernel<192> needs >= 128 tiles,
conv_halo_phase_kernel<192> >= 512 blocks, so the 64-128 px model tests never dispatch them).

* C4 cheng2020-attn q6 at 256x256: fp32 parity against the float64 oracle at B=1, and bf16 bounds at the
  per-GPU batch B=4 with conv_halo_s1_kernel<192> asserted in the step's launches;
* C2' bmshj2018-hyperprior q6 (192, 320) at 256x256, B=16, bf16, with conv_halo_phase_kernel<192> asserted;
* C5 at paper resolution (master.py:708-742, 158-210): Spatial_aligner on its three token
  grids (32x40, 64x80, 128x160) against the CPU oracle, Channel_aligner on 512x640 features against the
  oracle module run on the GPU in fp32 (torch's own convolutions: the CPU would take minutes for its ~7
  TFLOP), and one full training step of Master_compresser(512, 640) guided by Guided_compresser on
  1024x1280 RGB, B=2: bf16 loss within 2 % of the HIP fp32 step, finite gradients.

Bars as in test_models_wide_gpu.py (fp32: 1e-4 outputs / 2e-3 gradients against float64, or 2x the fp32
oracle's own error; bf16: x_hat 1e-2, likelihoods 2e-2, loss 1e-3, gradient cosine)."""
import math

import pytest
import torch

import cai_oracle as O
import cai_oracle_master as OM

pytestmark = pytest.mark.gpu


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    d = b.norm().item()
    return (a - b).norm().item() / (d if d > 0 else 1.0)


def _pair(name, args, dev):
    from compressai.zoo import model_architectures

    torch.manual_seed(0)
    ref = O.ARCHS[name](*args)
    net = model_architectures[name](*args)
    net.load_state_dict(ref.state_dict())
    return ref, net.to(dev)


def _run(name, args, size, batch, cuda, bf16, quality, seed):
    """Oracle (fp32 CPU) and HIP step on the same weights / input / noise; the HIP step under the ledger,
    so the kernels it launched are known."""
    from compressai import _ledger
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss

    ref, net = _pair(name, args, cuda)
    x = torch.rand(batch, 3, size, size, generator=torch.Generator().manual_seed(seed))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(seed + 1))
    with feed:
        out_r = ref(x)
    cr = O.RateDistortionLoss(quality)(out_r, x)
    cr["loss"].backward()
    q = [n.to(cuda) for n in feed.drawn]
    set_noise_source(lambda t: q.pop(0))
    try:
        with _ledger.recording(keep_replay=False) as led:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(x.to(cuda))
                c = RateDistortionLoss(quality)(out, x.to(cuda))
            c["loss"].backward()
            torch.cuda.synchronize()
    finally:
        set_noise_source(None)
    assert not q
    kernels = {e.kernel for e in led.entries}
    return ref, net, out_r, out, cr, c, feed.drawn, x, kernels


def test_cheng2020_attn_fp32_parity_256(cuda):
    name, args = "cheng2020-attn", (192,)
    ref, net, out_r, out, cr, c, drawn, x, _ = _run(name, args, 256, 1, cuda, False, 6, seed=31)
    import copy

    r64 = copy.deepcopy(ref).double()
    for p in r64.parameters():
        p.grad = None
    with O.NoiseFeed([n.double() for n in drawn]):
        out64 = r64(x.double())
    O.RateDistortionLoss(6)(out64, x.double())["loss"].backward()

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


BF16_XHAT, BF16_LIK, BF16_LOSS, GRAD_COS, TENSOR_COS = 1e-2, 2e-2, 1e-3, 0.9999, 0.98


@pytest.mark.parametrize("name,args,batch,quality,gated", [
    ("cheng2020-attn", (192,), 4, 6, "conv_halo_s1_kernel<192>"),                   # C4, per-GPU batch
    ("bmshj2018-hyperprior", (192, 320), 16, 6, "conv_halo_phase_kernel<192>"),      # C2' at C2's batch
], ids=["cheng2020-attn-q6-B4", "hyperprior-q6-B16"])
def test_bf16_production_mix_256(cuda, name, args, batch, quality, gated):
    ref, net, out_r, out, cr, c, _, _, kernels = _run(name, args, 256, batch, cuda, True, quality, seed=41)
    assert gated in kernels, sorted(kernels)
    ex = relerr(out["x_hat"], out_r["x_hat"])
    el = {k: relerr(out["likelihoods"][k], out_r["likelihoods"][k]) for k in out_r["likelihoods"]}
    eloss = abs(c["loss"].item() - cr["loss"].item()) / abs(cr["loss"].item())
    pr = dict(ref.named_parameters())
    tcos, dots, na, nb = {}, 0.0, 0.0, 0.0
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None or p.grad is None:
            continue
        g = p.grad.detach().float().cpu()
        assert torch.isfinite(g).all(), n
        tcos[n] = float(torch.nn.functional.cosine_similarity(g.double().flatten(), gr.double().flatten(), dim=0))
        dots += float((g.double() * gr.double()).sum())
        na += float((g.double() ** 2).sum())
        nb += float((gr.double() ** 2).sum())
    cos = dots / math.sqrt(na * nb)
    low = sorted(tcos.items(), key=lambda kv: kv[1])[:3]
    print(f"\nbf16 {name} B={batch}: x_hat {ex:.3e} lik {el} loss {eloss:.3e} grad cos {cos:.6f} lowest {low}")
    assert ex < BF16_XHAT
    for k, v in el.items():
        assert v < BF16_LIK, k
    assert eloss < BF16_LOSS
    assert cos > GRAD_COS
    assert low[0][1] > TENSOR_COS, low


# ---------------------------------------------------------------------------------------------------------
# C5 at paper resolution: IR 512x640 (channel 1, master stride 1), RGB 1024x1280 guide
# ---------------------------------------------------------------------------------------------------------

def _copy(ref, mod, cuda):
    mod.load_state_dict(ref.state_dict())
    return mod.to(cuda)


@pytest.mark.parametrize("res", [(64, 80), (128, 160), (256, 320)], ids=["tokens32x40", "tokens64x80",
                                                                       "tokens128x160"])
def test_spatial_aligner_paper_grids(cuda, res):
    """Master_decoder(width=512, height=640).sp_aligner{1,2,3}: inputs (64, 80), (128, 160), (256, 320),
    i.e. Swin token grids 32x40, 64x80, 128x160 (window 4, shift 0 / 2), fp32 B=1 vs the CPU oracle."""
    from compressai.models.master import Spatial_aligner

    torch.manual_seed(50 + res[0])
    ref = OM.Spatial_aligner(input_resolution=res)
    with torch.no_grad():
        for blk in ref.blocks:
            blk.attn.relative_position_bias_table.normal_(0, 0.5)
    mod = _copy(ref, Spatial_aligner(input_resolution=res), cuda)
    gen = torch.Generator().manual_seed(60 + res[0])
    x = torch.randn(1, 192, *res, generator=gen)
    gd = torch.randn(1, 192, *res, generator=gen)
    xr, gr = x.clone().requires_grad_(), gd.clone().requires_grad_()
    yr = ref(xr, gr)
    g = torch.randn(yr.shape, generator=gen)
    yr.backward(g)
    xd = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    gdd = gd.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = mod(xd, gdd)
    y.backward(g.to(cuda))
    assert relerr(y, yr) < 1e-4
    assert relerr(xd.grad, xr.grad) < 2e-3
    assert relerr(gdd.grad, gr.grad) < 2e-3
    pr = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert relerr(p.grad, pr[n].grad) < 2e-3, n


def test_channel_aligner_512x640(cuda):
    """Channel_aligner (4 x conv3x3(256) trunk per branch, conv5/conv6 heads, global pools) on the IR
    config's 64-channel 512x640 features, fp32 B=1, against the oracle module on the GPU in fp32."""
    from compressai.models.master import Channel_aligner

    prev = (torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    try:
        torch.manual_seed(70)
        ref = OM.Channel_aligner()
        mod = _copy(ref, Channel_aligner(), cuda)
        ref = ref.to(cuda)
        gen = torch.Generator().manual_seed(71)
        f1 = torch.randn(1, 64, 512, 640, generator=gen)
        f2 = torch.randn(1, 64, 512, 640, generator=gen)
        g = torch.randn(1, 64, 512, 640, generator=gen).to(cuda)
        r1, r2 = f1.to(cuda).requires_grad_(), f2.to(cuda).requires_grad_()
        out_r, beta_r, gamma_r = ref(r1, r2)
        (out_r * g).sum().backward()
        d1 = f1.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
        d2 = f2.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
        out, beta, gamma = mod(d1, d2)
        (out * g).sum().backward()
        errs = {"out": (relerr(out, out_r), rel_l2(out, out_r)), "beta": (relerr(beta, beta_r), rel_l2(beta, beta_r)),
                "gamma": (relerr(gamma, gamma_r), rel_l2(gamma, gamma_r)),
                "d1": (relerr(d1.grad, r1.grad), rel_l2(d1.grad, r1.grad)),
                "d2": (relerr(d2.grad, r2.grad), rel_l2(d2.grad, r2.grad))}
        pr = dict(ref.named_parameters())
        for n, p in mod.named_parameters():
            errs[n] = (relerr(p.grad, pr[n].grad), rel_l2(p.grad, pr[n].grad))
        print("\nChannel_aligner 512x640 (max, rel-L2):", {k: (f"{a:.2e}", f"{b:.2e}") for k, (a, b) in errs.items()})
        for k in ("out", "beta", "gamma"):
            assert errs[k][0] < 1e-4, (k, errs[k])
        for k, (emax, el2) in errs.items():
            assert el2 < 1e-4, (k, emax, el2)
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = prev


def test_master_guided_full_resolution_step(cuda):
    """BASELINE configs[4] per GPU: Master_compresser(width=512, height=640, channel=1) on IR 512x640 guided
    by Guided_compresser(channel=3) on RGB 1024x1280 (no_grad, training mode), B=2, one RD-loss training
    step in bf16 autocast and in the HIP fp32 mode on the same weights and noise: shapes, finite loss and
    gradients, bf16 loss within 2 % of fp32, bf16 gradient cosine against fp32."""
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.models import Guided_compresser, Master_compresser

    torch.manual_seed(80)
    net = Master_compresser(width=512, height=640, channel=1).to(cuda).train()
    guide = Guided_compresser(channel=3).to(cuda).train()
    gen = torch.Generator().manual_seed(81)
    x = torch.rand(2, 1, 512, 640, generator=gen).to(cuda)
    gx = torch.rand(2, 3, 1024, 1280, generator=gen).to(cuda)
    drawn = []
    ngen = torch.Generator().manual_seed(82)

    def record(t):
        n = torch.empty(t.shape).uniform_(-0.5, 0.5, generator=ngen).to(cuda)
        drawn.append(n)
        return n

    def step(bf16, source):
        net.zero_grad(set_to_none=True)
        set_noise_source(source)
        try:
            with torch.no_grad():
                hidden = guide(gx)["hidden"]
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(x, gx, hidden)
                c = RateDistortionLoss(1)(out, x)
            c["loss"].backward()
        finally:
            set_noise_source(None)
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().float().clone() for n, p in net.named_parameters() if p.grad is not None}
        return out, c, hidden, grads

    out32, c32, hidden, g32 = step(False, record)
    assert out32["x_hat"].shape == (2, 1, 512, 640)
    assert out32["likelihoods"]["y"].shape == (2, 192, 32, 40)
    assert out32["likelihoods"]["z"].shape == (2, 192, 8, 10)
    assert hidden["gs1"].shape == (2, 192, 128, 160) and hidden["gs3"].shape == (2, 192, 512, 640)
    replay = list(drawn)
    out16, c16, _, g16 = step(True, lambda t: replay.pop(0))
    assert not replay
    l32, l16 = c32["loss"].item(), c16["loss"].item()
    assert math.isfinite(l32) and math.isfinite(l16)
    assert abs(l16 - l32) < 0.02 * abs(l32), (l16, l32)
    assert set(g16) == set(g32) and not any(n.startswith("g_s.") for n in g32)   # inherited g_s unused
    dots = na = nb = 0.0
    for n in g32:
        assert torch.isfinite(g16[n]).all() and torch.isfinite(g32[n]).all(), n
        dots += float((g16[n].double() * g32[n].double()).sum())
        na += float((g16[n].double() ** 2).sum())
        nb += float((g32[n].double() ** 2).sum())
    cos = dots / math.sqrt(na * nb)
    print(f"\nC5 full resolution: loss fp32 {l32:.5f} bf16 {l16:.5f}, gradient cosine {cos:.6f}")
    assert cos > 0.999
