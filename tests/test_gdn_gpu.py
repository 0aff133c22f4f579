"""GDN family beyond the benchmarked widths: GDN1 (layers/gdn.py:95-121) and GDN / IGDN at channel counts other
than the models' N (the reference layer takes any C, gdn.py:41-92), against the CPU oracle in exact fp32 and
with bf16 bounds."""
import pytest
import torch

import cai_oracle as O

pytestmark = pytest.mark.gpu


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def _pair(cls_o, cls_p, C, inverse, dev, seed=0):
    torch.manual_seed(seed)
    ref = cls_o(C, inverse=inverse)
    with torch.no_grad():   # a non-trivial gamma / beta (not the identity init)
        ref.gamma.add_(0.05 * torch.rand(C, C))
        ref.beta.add_(0.1 * torch.rand(C))
    net = cls_p(C, inverse=inverse)
    net.load_state_dict(ref.state_dict())
    return ref, net.to(dev)


def _run(ref, net, x, g, dev, bf16=False):
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g)
    xd = x.to(dev).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
        yd = net(xd)
    yd.backward(g.to(dev).to(yd.dtype))
    return xr, yr, xd, yd


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("C", [16, 40, 64])
def test_gdn1_fp32_matches_oracle(cuda, C, inverse):
    from compressai.layers import GDN1

    ref, net = _pair(O.GDN1, GDN1, C, inverse, cuda)
    x = torch.randn(2, C, 9, 11, generator=torch.Generator().manual_seed(1))
    g = torch.randn(2, C, 9, 11, generator=torch.Generator().manual_seed(2))
    xr, yr, xd, yd = _run(ref, net, x, g, cuda)
    assert relerr(yd, yr) < 1e-5
    assert relerr(xd.grad, xr.grad) < 1e-4
    assert relerr(net.beta.grad, ref.beta.grad) < 1e-4
    assert relerr(net.gamma.grad, ref.gamma.grad) < 1e-4


def test_gdn1_bf16_is_close(cuda):
    from compressai.layers import GDN1

    ref, net = _pair(O.GDN1, GDN1, 128, False, cuda)
    x = torch.randn(2, 128, 16, 16, generator=torch.Generator().manual_seed(3))
    g = torch.randn(2, 128, 16, 16, generator=torch.Generator().manual_seed(4))
    xr, yr, xd, yd = _run(ref, net, x, g, cuda, bf16=True)
    assert relerr(yd, yr) < 2e-2
    assert relerr(xd.grad, xr.grad) < 3e-2
    cos = torch.nn.functional.cosine_similarity(net.gamma.grad.cpu().flatten(), ref.gamma.grad.flatten(), dim=0)
    assert cos > 0.999


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("C", [16, 48, 96, 160, 192])
def test_gdn_any_width_fp32_matches_oracle(cuda, C, inverse):
    """Widths off the models' N: multiples of 32 run natively, others through the zero-padded path."""
    from compressai.layers import GDN

    ref, net = _pair(O.GDN, GDN, C, inverse, cuda)
    x = torch.randn(2, C, 7, 13, generator=torch.Generator().manual_seed(5))
    g = torch.randn(2, C, 7, 13, generator=torch.Generator().manual_seed(6))
    xr, yr, xd, yd = _run(ref, net, x, g, cuda)
    assert relerr(yd, yr) < 1e-5
    assert relerr(xd.grad, xr.grad) < 1e-4
    assert relerr(net.beta.grad, ref.beta.grad) < 1e-4
    assert relerr(net.gamma.grad, ref.gamma.grad) < 1e-4


@pytest.mark.parametrize("C", [72, 224, 256])
def test_gdn_wide_bf16_is_close(cuda, C):
    from compressai.layers import GDN

    ref, net = _pair(O.GDN, GDN, C, False, cuda)
    x = torch.randn(2, C, 16, 16, generator=torch.Generator().manual_seed(7))
    g = torch.randn(2, C, 16, 16, generator=torch.Generator().manual_seed(8))
    xr, yr, xd, yd = _run(ref, net, x, g, cuda, bf16=True)
    assert relerr(yd, yr) < 2e-2
    assert relerr(xd.grad, xr.grad) < 3e-2
    cos = torch.nn.functional.cosine_similarity(net.gamma.grad.cpu().flatten(), ref.gamma.grad.flatten(), dim=0)
    assert cos > 0.999


def test_gdn_too_wide_raises(cuda):
    from compressai.layers import GDN

    net = GDN(300).to(cuda)
    with pytest.raises(ValueError, match="supports up to"):
        net(torch.rand(1, 300, 4, 4, device=cuda))
