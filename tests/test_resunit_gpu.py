"""The fused ResidualUnit kernel (csrc/resunit.hip, cai_resunit) against a float32 torch restatement of
layers.py:211-226 on the same bf16 operands, and the fused chain against the per-conv chain at model level.

Forward: h1 = relu(conv1x1_a(x) + ba), h2 = relu(conv3x3_b(h1) + bb), y = relu(conv1x1_c(h2) + bc + x), each
rounded to bf16 as the kernel stores it; the reference takes the kernel's own bf16 h1 / h2 as the next layer's
input, so every comparison is one layer's bf16 rounding deep.  Backward: the reference applies the kernel's saved
masks (y, h2, h1 > 0) to the same bf16 gradients.  Bars: 1e-2 relative (max-norm) per tensor -- bf16 output
rounding (2^-8) plus fp32 accumulation-order differences.  Sizes cover ragged 8x8 tiles (13 x 21), the image
border (zero padding of h1), both channel counts and the masked / unmasked output-gradient modes.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def relerr(a, b):
    a, b = a.float(), b.float()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def _weights(n, dev, seed):
    g = torch.Generator().manual_seed(seed)
    nh = n // 2
    wa = torch.randn(nh, n, 1, 1, generator=g) / n ** 0.5
    wb = torch.randn(nh, nh, 3, 3, generator=g) / (9 * nh) ** 0.5
    wc = torch.randn(n, nh, 1, 1, generator=g) / nh ** 0.5
    ba, bb, bc = (0.1 * torch.randn(c, generator=g) for c in (nh, nh, n))
    return [t.to(dev) for t in (wa, ba, wb, bb, wc, bc)]


def _pm(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("n,B,H,W", [(192, 2, 16, 16), (192, 1, 13, 21), (128, 2, 9, 16), (128, 1, 8, 8)])
@pytest.mark.parametrize("gy_masked", [False, True])
def test_resunit_kernel_vs_torch(cuda, n, B, H, W, gy_masked):
    from compressai import _ops

    torch.manual_seed(n + H)
    wa, ba, wb, bb, wc, bc = _weights(n, cuda, n + W)
    x = _pm(torch.randn(B, n, H, W, device=cuda)).to(torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, u = _ops._resunit_fwd(x, (wa, ba, wb, bb, wc, bc), True)
    torch.cuda.synchronize()
    xpm, h1, h2, yk = u.saved_tensors
    r = lambda t: t.to(torch.bfloat16).float()    # noqa: E731  (bf16 weights, as packed)
    h1r = F.relu(F.conv2d(x.float(), r(wa), ba))
    h2r = F.relu(F.conv2d(h1.float(), r(wb), bb, padding=1))
    yr = F.relu(F.conv2d(h2.float(), r(wc), bc) + x.float())
    assert relerr(h1, h1r) < 1e-2 and relerr(h2, h2r) < 1e-2 and relerr(y, yr) < 1e-2

    gy = _pm(torch.randn(B, n, H, W, device=cuda)).to(torch.bfloat16)
    if gy_masked:
        gy = (gy.float() * (y.float() > 0)).to(torch.bfloat16)
    u.gy_masked = gy_masked
    res2 = _pm(torch.randn(B, n, H, W, device=cuda)).to(torch.bfloat16)
    u.dx_res2 = res2
    u.mask_x = True
    grads = {}
    real = _ops.conv_wgrad

    def spy(g, dt, xpm_, xld, in_abs, gpm, gld, wparam, bparam, weight, has_bias):
        grads[id(wparam)] = (xpm_, gpm)
        return real(g, dt, xpm_, xld, in_abs, gpm, gld, wparam, bparam, weight, has_bias)

    _ops.conv_wgrad = spy
    try:
        dx, pg = _ops._resunit_bwd(u, gy)
    finally:
        _ops.conv_wgrad = real
    torch.cuda.synchronize()
    gc = gy.float() * (y.float() > 0)
    gbr = F.conv2d(gc, r(wc).transpose(0, 1)) * (h2.float() > 0)
    gb = grads[id(wb)][1]
    assert relerr(gb, gbr) < 1e-2
    gar = F.conv_transpose2d(gb.float(), r(wb), padding=1) * (h1.float() > 0)
    ga = grads[id(wa)][1]
    assert relerr(ga, gar) < 1e-2
    dxr = (F.conv2d(ga.float(), r(wa).transpose(0, 1)) + gc + res2.float()) * (x.float() > 0)
    assert relerr(dx, dxr) < 1e-2
    if not gy_masked:
        assert relerr(grads[id(wc)][1], gc) < 1e-2
    # the weight gradients come from the kernel's tensors through the conv wgrad path
    dwa = pg[0]
    dwar = torch.einsum("bchw,bkhw->kc", x.float(), ga.float()).reshape(wa.shape)
    assert relerr(dwa, dwar) < 2e-2


@pytest.mark.parametrize("n,H", [(192, 64), (192, 16), (128, 32)])
def test_attention_block_fused_units_vs_per_conv(cuda, n, H):
    """AttentionBlock (layers.py:196-244) with its six ResidualUnits on the fused kernel against the per-conv
    chain (CAI_RESUNIT_FUSED=0 path) on the same weights and input: output, input gradient, every parameter
    gradient (bf16 bars: relative max-norm 2e-2, cosine >= 0.999)."""
    import compressai.layers as L
    from compressai import _ops

    torch.manual_seed(H)
    mod = L.AttentionBlock(n).to(cuda)
    x0 = _pm(torch.randn(2, n, H, H, device=cuda))
    gy = _pm(torch.randn(2, n, H, H, device=cuda))
    outs = {}
    for fused in (False, True):
        _ops._RESUNIT_FUSED = fused
        try:
            mod.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(x)
            (y.float() * gy).sum().backward()
            torch.cuda.synchronize()
            outs[fused] = (y.float().detach(), x.grad.float(), {k: p.grad.float().clone() for k, p in
                                                                  mod.named_parameters()})
        finally:
            _ops._RESUNIT_FUSED = True
    (ya, dxa, ga), (yb, dxb, gb) = outs[False], outs[True]
    assert relerr(yb, ya) < 2e-2
    assert relerr(dxb, dxa) < 2e-2
    for k in ga:
        cos = torch.nn.functional.cosine_similarity(ga[k].flatten(), gb[k].flatten(), dim=0).item()
        assert cos > 0.999, (k, cos)


def test_resunit_launch_count(cuda, monkeypatch):
    """One AttentionBlock step on the fused path: 6 cai_resunit forwards and 6 backwards, no per-conv residual
    launches left."""
    import compressai.layers as L
    from compressai import _ops

    calls = []
    real = _ops.lib

    class Spy:
        def __getattr__(self, name):
            fn = getattr(real, name)
            if not name.startswith(("cai_resunit", "cai_conv_fwd_res", "cai_conv_dgrad_res")):
                return fn

            def call(*a):
                calls.append((name, a[1] if name == "cai_resunit" else None))
                return fn(*a)
            return call

    monkeypatch.setattr(_ops, "lib", Spy())
    mod = L.AttentionBlock(192).to(cuda)
    x = _pm(torch.randn(1, 192, 16, 16, device=cuda)).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = mod(x)
    y.float().sum().backward()
    torch.cuda.synchronize()
    names = [c[0] for c in calls]
    assert names.count("cai_resunit") == 12, calls
    assert sum(1 for c in calls if c[0] == "cai_resunit" and c[1] == 1) == 6
    assert not any(n.startswith("cai_conv_fwd_res") or n.startswith("cai_conv_dgrad_res") for n in names)
