"""Stride-2 image-side layers on the space-to-depth kernels (csrc/edge.hip) vs plain PyTorch fp32.

The edge path computes in bf16 (operands rounded once, fp32 accumulation), so the reference here is
torch fp32 on the same bf16-rounded operands: what remains is summation order and the bf16 rounding
of bf16 outputs.  Tolerance: relative max error <= 1e-2 (outputs, dx, dW, db).  The general
implicit-GEMM path (CAI_EDGE_OFF) must agree to the same tolerance.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 1e-2


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


def _bf(t):
    return t.bfloat16().float()


CONV = [  # B, C, N, H, W, k  (image H x W, feature grid H/2 x W/2)
    (2, 3, 128, 64, 64, 5),
    (2, 3, 192, 48, 80, 5),
    (2, 1, 128, 32, 34, 3),
    (3, 2, 192, 20, 132, 1),
    (2, 3, 128, 256, 256, 5),
    (8, 3, 128, 256, 256, 5),     # more tiles than resident blocks: several tiles per persistent block
    (6, 3, 192, 200, 330, 5),     # ragged column blocks, several tiles per block
]
DECONV = [  # B, N, C, H, W, k  (feature grid H x W, image 2H x 2W)
    (2, 128, 3, 32, 32, 5),
    (2, 192, 3, 20, 33, 5),
    (2, 128, 1, 17, 70, 3),
    (1, 128, 3, 128, 128, 5),
    (4, 128, 3, 128, 128, 5),     # input-gradient tiles > resident blocks
]


def _supported(cin, cout, k, transposed, B, H, W):
    import ctypes

    from compressai._native import BF16, ConvGeom, lib

    if transposed:
        g = ConvGeom(B, cin, H, W, cout, 2 * H, 2 * W, k, 2, k // 2, 1, 1)
    else:
        g = ConvGeom(B, cin, H, W, cout, H // 2, W // 2, k, 2, k // 2, 0, 0)
    return lib.cai_edge_supported(ctypes.byref(g), BF16) == 1


@pytest.mark.parametrize("case", CONV, ids=[f"conv{c[1]}-{c[2]}k{c[5]}_{c[3]}x{c[4]}" for c in CONV])
def test_edge_conv(cuda, case):
    from compressai import _ops
    from compressai.layers import Conv2d

    B, C, N, H, W, k = case
    assert _supported(C, N, k, False, B, H, W)
    torch.manual_seed(0)
    ref = nn.Conv2d(C, N, k, stride=2, padding=k // 2)
    mod = Conv2d(C, N, k, stride=2, padding=k // 2)
    mod.load_state_dict(ref.state_dict())
    mod = mod.to(cuda)
    x = torch.rand(B, C, H, W)
    g = torch.randn(B, N, H // 2, W // 2)
    wr = _bf(ref.weight.detach()).requires_grad_()
    br = ref.bias.detach().clone().requires_grad_()
    yr = F.conv2d(_bf(x), wr, br, stride=2, padding=k // 2)
    yr.backward(_bf(g))
    outs = {}
    for off in (False, True):
        _ops._EDGE_OFF = off
        try:
            mod.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(x.to(cuda))
            y.backward(g.to(cuda))
            outs[off] = (y.float(), mod.weight.grad.clone(), mod.bias.grad.clone())
        finally:
            _ops._EDGE_OFF = False
    y, dw, db = outs[False]
    assert y.shape == yr.shape
    assert relerr(y, yr) < TOL
    assert relerr(dw, wr.grad) < TOL
    assert relerr(db, br.grad) < TOL
    for a, b in zip(outs[False], outs[True]):
        assert relerr(a, b) < TOL


@pytest.mark.parametrize("case", DECONV, ids=[f"deconv{c[1]}-{c[2]}k{c[5]}_{c[3]}x{c[4]}" for c in DECONV])
def test_edge_deconv(cuda, case):
    from compressai import _ops
    from compressai.layers import ConvTranspose2d

    B, N, C, H, W, k = case
    assert _supported(N, C, k, True, B, H, W)
    torch.manual_seed(1)
    ref = nn.ConvTranspose2d(N, C, k, stride=2, padding=k // 2, output_padding=1)
    mod = ConvTranspose2d(N, C, k, stride=2, padding=k // 2, output_padding=1)
    mod.load_state_dict(ref.state_dict())
    mod = mod.to(cuda)
    x = torch.randn(B, N, H, W)
    g = torch.randn(B, C, 2 * H, 2 * W)
    xr = _bf(x).requires_grad_()
    wr = _bf(ref.weight.detach()).requires_grad_()
    br = ref.bias.detach().clone().requires_grad_()
    yr = F.conv_transpose2d(xr, wr, br, stride=2, padding=k // 2, output_padding=1)
    yr.backward(_bf(g))
    outs = {}
    for off in (False, True):
        _ops._EDGE_OFF = off
        try:
            mod.zero_grad(set_to_none=True)
            xd = x.to(cuda).requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(xd)
            y.backward(g.to(cuda))
            outs[off] = (y.float(), xd.grad.float(), mod.weight.grad.clone(), mod.bias.grad.clone())
        finally:
            _ops._EDGE_OFF = False
    y, dx, dw, db = outs[False]
    assert y.shape == yr.shape and y.dtype == torch.float32
    assert relerr(y, yr) < TOL
    assert relerr(dx, xr.grad) < TOL
    assert relerr(dw, wr.grad) < TOL
    assert relerr(db, g.sum((0, 2, 3))) < 1e-4      # fp32 column sums of dy
    for a, b in zip(outs[False], outs[True]):
        assert relerr(a, b) < TOL


def test_edge_grads_accumulate(cuda):
    """Two backward passes accumulate into .grad (the direct-gradient path of the optimizer buffers is
    the same kernel with accumulate=1)."""
    from compressai.layers import Conv2d

    torch.manual_seed(2)
    mod = Conv2d(3, 128, 5, stride=2, padding=2).to(cuda)
    x = torch.rand(2, 3, 32, 32, device=cuda)
    for _ in range(2):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = mod(x)
        y.float().sum().backward()
    w1 = mod.weight.grad.clone()
    mod.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = mod(x)
    y.float().sum().backward()
    assert relerr(w1, 2 * mod.weight.grad) < 1e-5
