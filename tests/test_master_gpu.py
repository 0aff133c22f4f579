"""Multi-modal codec (compressai/models/master.py): HIP path vs the CPU oracle
(oracle/cai_oracle_master.py) on identical weights, inputs and injected noise.

fp32 mode: outputs within 1e-4 relative (likelihoods, x_hat), gradients within
2e-3 relative.  bf16 mode: the error against the fp32 oracle stays within 2x
(+1 %) of PyTorch's own bf16 autocast on the same GPU.
"""
import pytest
import torch

import cai_oracle as O
import cai_oracle_master as OM

pytestmark = pytest.mark.gpu


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def _grad_check(net, ref, tol=2e-3):
    """Per-tensor relative error, with the denominator floored at 1e-6 of the largest
    gradient in the model (tensors whose true gradient is round-off noise)."""
    pr = dict(ref.named_parameters())
    gmax = max(p.grad.abs().max().item() for p in ref.parameters() if p.grad is not None)
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None:
            assert p.grad is None or p.grad.abs().max().item() == 0, n
            continue
        den = max(gr.abs().max().item(), 1e-6 * gmax)
        err = (p.grad.detach().float().cpu() - gr).abs().max().item() / den
        assert err < tol, (n, err)


def _copy(ref, mod, cuda):
    mod.load_state_dict(ref.state_dict())
    return mod.to(cuda)


def _tokens(B, C, H, W, seed):
    return torch.randn(B, C, H, W, generator=torch.Generator().manual_seed(seed))


def _ref_tokens(t):
    """pixel-major logical [B, C, H, W] -> the oracle's (B, L, C) token tensor."""
    return t.flatten(2).transpose(1, 2).contiguous()


@pytest.mark.parametrize("C,H,W", [(96, 8, 12), (64, 8, 12), (192, 8, 12), (96, 128, 160)],
                         ids=["96", "64", "192-general", "96-40960tok"])
def test_layernorm(cuda, C, H, W):
    """LayerNorm fwd / bwd against torch fp32.  C <= 128 runs the register backward, 192 the general one; 40960
    tokens (the multimodal Swin blocks' largest map) give 640 partial blocks for the parameter-gradient reduce."""
    from compressai.models.master import LayerNorm

    torch.manual_seed(0)
    ref = torch.nn.LayerNorm(C)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.5, 0.5)
    mod = _copy(ref, LayerNorm(C), cuda)
    x = _tokens(2, C, H, W, 1)
    g = _tokens(2, C, H, W, 2)
    xr = _ref_tokens(x).requires_grad_()
    yr = ref(xr)
    yr.backward(_ref_tokens(g))
    xd = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = mod(xd)
    y.backward(g.to(cuda))
    assert relerr(_ref_tokens(y), yr) < 1e-5
    assert relerr(_ref_tokens(xd.grad), xr.grad) < 1e-4
    assert relerr(mod.weight.grad, ref.weight.grad) < 1e-4
    assert relerr(mod.bias.grad, ref.bias.grad) < 1e-4


def test_gelu(cuda):
    from compressai.models.master import GELU

    x = _tokens(2, 64, 4, 4, 3) * 3
    g = _tokens(2, 64, 4, 4, 4)
    xr = x.clone().requires_grad_()
    yr = torch.nn.GELU()(xr)
    yr.backward(g)
    xd = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = GELU()(xd)
    y.backward(g.to(cuda))
    assert relerr(y, yr) < 1e-6
    assert relerr(xd.grad, xr.grad) < 1e-5


def test_gelu_and_channel_affine_bf16(cuda):
    """The bf16 8-channel-chunk kernels (GELU fwd / bwd, the channel aligner's y = gamma * x + beta and its input
    gradient) against torch fp32 on the same bf16 operands: relative max 1e-2 (one bf16 rounding of the output)."""
    from compressai._ops import ChannelAffineFn
    from compressai.models.master import GELU

    torch.manual_seed(21)
    x = (torch.randn(2, 96, 16, 20, device=cuda) * 3).bfloat16().contiguous(memory_format=torch.channels_last)
    g = torch.randn(2, 96, 16, 20, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    xd = x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = GELU()(xd)
    y.backward(g)
    xr = x.float().requires_grad_()
    yr = torch.nn.GELU()(xr)
    yr.backward(g.float())
    assert relerr(y.float(), yr) < 1e-2
    assert relerr(xd.grad.float(), xr.grad) < 1e-2

    f = torch.randn(2, 64, 24, 20, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    gamma = torch.randn(2, 64, 1, 1, device=cuda, requires_grad=True)
    beta = torch.randn(2, 64, 1, 1, device=cuda, requires_grad=True)
    fd = f.clone().requires_grad_()
    gy = torch.randn(2, 64, 24, 20, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = ChannelAffineFn.apply(fd, gamma, beta)
    out.backward(gy)
    fr = f.float().requires_grad_()
    gr, br = gamma.detach().clone().requires_grad_(), beta.detach().clone().requires_grad_()
    outr = gr * fr + br
    outr.backward(gy.float())
    assert relerr(out.float(), outr) < 1e-2
    assert relerr(fd.grad.float(), fr.grad) < 1e-2
    assert relerr(gamma.grad, gr.grad) < 1e-2 and relerr(beta.grad, br.grad) < 1e-2


@pytest.mark.parametrize("shift", [0, 2])
@pytest.mark.parametrize("res", [(8, 8), (8, 12), (12, 8)])
def test_swin_block(cuda, shift, res):
    """SwinTransformerBlock (cross attention, rel-pos bias, shifted-window mask) fwd + bwd."""
    from compressai.models.master import SwinTransformerBlock

    torch.manual_seed(5)
    ref = OM.SwinTransformerBlock(dim=96, input_resolution=res, num_heads=3, window_size=4, shift_size=shift)
    with torch.no_grad():
        ref.attn.relative_position_bias_table.normal_(0, 0.5)
    mod = _copy(ref, SwinTransformerBlock(dim=96, input_resolution=res, num_heads=3, window_size=4,
                                          shift_size=shift), cuda)
    H, W = res
    x = _tokens(2, 96, H, W, 6)
    gd = _tokens(2, 96, H, W, 7)
    g = _tokens(2, 96, H, W, 8)
    xr, gr = _ref_tokens(x).requires_grad_(), _ref_tokens(gd).requires_grad_()
    yr = ref(xr, gr)
    yr.backward(_ref_tokens(g))
    xd = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    gdd = gd.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = mod(xd, gdd)
    y.backward(g.to(cuda))
    assert relerr(_ref_tokens(y), yr) < 1e-4
    assert relerr(_ref_tokens(xd.grad), xr.grad) < 2e-3
    assert relerr(_ref_tokens(gdd.grad), gr.grad) < 2e-3
    pr = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert relerr(p.grad, pr[n].grad) < 2e-3, n


def test_spatial_aligner(cuda):
    from compressai.models.master import Spatial_aligner

    torch.manual_seed(9)
    ref = OM.Spatial_aligner(input_resolution=(16, 24))
    mod = _copy(ref, Spatial_aligner(input_resolution=(16, 24)), cuda)
    x = torch.randn(2, 192, 16, 24, generator=torch.Generator().manual_seed(10))
    gd = torch.randn(2, 192, 16, 24, generator=torch.Generator().manual_seed(11))
    xr, gr = x.clone().requires_grad_(), gd.clone().requires_grad_()
    yr = ref(xr, gr)
    g = torch.randn(yr.shape, generator=torch.Generator().manual_seed(12))
    yr.backward(g)
    xd, gdd = x.to(cuda).requires_grad_(), gd.to(cuda).requires_grad_()
    y = mod(xd, gdd)
    y.backward(g.to(cuda))
    assert relerr(y, yr) < 1e-4
    assert relerr(xd.grad, xr.grad) < 2e-3
    assert relerr(gdd.grad, gr.grad) < 2e-3
    pr = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert relerr(p.grad, pr[n].grad) < 2e-3, n


def test_channel_aligner(cuda):
    from compressai.models.master import Channel_aligner

    torch.manual_seed(13)
    ref = OM.Channel_aligner()
    mod = _copy(ref, Channel_aligner(), cuda)
    f1 = torch.randn(2, 64, 12, 10, generator=torch.Generator().manual_seed(14))
    f2 = torch.randn(2, 64, 12, 10, generator=torch.Generator().manual_seed(15))
    r1, r2 = f1.clone().requires_grad_(), f2.clone().requires_grad_()
    out_r, beta_r, gamma_r = ref(r1, r2)
    g = torch.randn(out_r.shape, generator=torch.Generator().manual_seed(16))
    (out_r * g).sum().backward()
    d1, d2 = f1.to(cuda).requires_grad_(), f2.to(cuda).requires_grad_()
    out, beta, gamma = mod(d1, d2)
    (out * g.to(cuda)).sum().backward()
    assert relerr(out, out_r) < 1e-4
    assert relerr(beta, beta_r) < 1e-4 and relerr(gamma, gamma_r) < 1e-4
    assert relerr(d1.grad, r1.grad) < 2e-3
    assert relerr(d2.grad, r2.grad) < 2e-3
    pr = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert relerr(p.grad, pr[n].grad) < 2e-3, n


def _noise_run(net, feed_drawn, cuda, *args):
    from compressai.entropy_models import set_noise_source

    q = [n.to(cuda) for n in feed_drawn]
    set_noise_source(lambda t: q.pop(0))
    try:
        return net(*args)
    finally:
        set_noise_source(None)


@pytest.mark.parametrize("channel", [3, 1])
def test_guided_compresser_train(cuda, channel):
    from compressai.losses import RateDistortionLoss
    from compressai.models import Guided_compresser

    torch.manual_seed(17)
    ref = OM.Guided_compresser(channel=channel)
    net = _copy(ref, Guided_compresser(channel=channel), cuda)
    x = torch.rand(1, channel, 128, 128, generator=torch.Generator().manual_seed(18))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(19))
    with feed:
        out_r = ref(x)
    cr = O.RateDistortionLoss(2)(out_r, x)
    cr["loss"].backward()
    out = _noise_run(net, feed.drawn, cuda, x.to(cuda))
    c = RateDistortionLoss(2)(out, x.to(cuda))
    c["loss"].backward()
    assert relerr(out["x_hat"], out_r["x_hat"]) < 1e-4
    for k in ("y", "z"):
        assert relerr(out["likelihoods"][k], out_r["likelihoods"][k]) < 1e-4, k
    for k in out_r["hidden"]:
        assert relerr(out["hidden"][k], out_r["hidden"][k]) < 1e-4, k
    assert abs(c["loss"].item() - cr["loss"].item()) <= 1e-4 * abs(cr["loss"].item())
    _grad_check(net, ref)


@pytest.mark.parametrize("channel", [1, 3])
def test_master_compresser_train(cuda, channel):
    """train.py:208-246 step body: guided under no_grad, master forward + RD loss + backward."""
    from compressai.losses import RateDistortionLoss
    from compressai.models import Master_compresser

    torch.manual_seed(20)
    guided_chl = 3 if channel == 1 else 1
    ref = OM.Master_compresser(width=64, height=64, channel=channel)
    net = _copy(ref, Master_compresser(width=64, height=64, channel=channel), cuda)
    refG = OM.Guided_compresser(channel=guided_chl).eval()
    if channel == 1:
        x = torch.rand(1, 1, 64, 64, generator=torch.Generator().manual_seed(21))
        gin = torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(22))
    else:
        x = torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(21))
        gin = torch.rand(1, 1, 64, 64, generator=torch.Generator().manual_seed(22))
    with torch.no_grad():
        hidden = refG(gin)["hidden"]
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(23))
    with feed:
        out_r = ref(x, gin, hidden)
    cr = O.RateDistortionLoss(2)(out_r, x)
    cr["loss"].backward()
    hd = {k: v.to(cuda) for k, v in hidden.items()}
    out = _noise_run(net, feed.drawn, cuda, x.to(cuda), gin.to(cuda), hd)
    c = RateDistortionLoss(2)(out, x.to(cuda))
    c["loss"].backward()
    assert relerr(out["x_hat"], out_r["x_hat"]) < 1e-4
    for k in ("y", "z"):
        assert relerr(out["likelihoods"][k], out_r["likelihoods"][k]) < 1e-4, k
    assert abs(c["loss"].item() - cr["loss"].item()) <= 1e-4 * abs(cr["loss"].item())
    _grad_check(net, ref)


def test_master_bf16_close(cuda):
    """bf16 autocast training forward: loss within 2 % of the fp32 oracle."""
    from compressai.losses import RateDistortionLoss
    from compressai.models import Master_compresser

    torch.manual_seed(24)
    ref = OM.Master_compresser(width=64, height=64, channel=1)
    net = _copy(ref, Master_compresser(width=64, height=64, channel=1), cuda)
    refG = OM.Guided_compresser(channel=3).eval()
    x = torch.rand(2, 1, 64, 64, generator=torch.Generator().manual_seed(25))
    gin = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(26))
    with torch.no_grad():
        hidden = refG(gin)["hidden"]
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(27))
    with feed:
        cr = O.RateDistortionLoss(2)(ref(x, gin, hidden), x)
    hd = {k: v.to(cuda) for k, v in hidden.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = _noise_run(net, feed.drawn, cuda, x.to(cuda), gin.to(cuda), hd)
        c = RateDistortionLoss(2)(out, x.to(cuda))
    c["loss"].backward()
    assert abs(c["loss"].item() - cr["loss"].item()) < 0.02 * abs(cr["loss"].item())
    assert all(torch.isfinite(p.grad).all() for p in net.parameters() if p.grad is not None)
