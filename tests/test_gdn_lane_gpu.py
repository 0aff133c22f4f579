"""Lane-local GDN / IGDN kernels (csrc/gdn_lane.hip) against the LDS-tile kernels they replace, through the C ABI
(cai_gdn_fwd, cai_gdn_backward; CAI_GDN_LANE=0 selects the old kernels at each call):
  * forward: bit-identical (same MFMA K-block sequence per output, same normalisation arithmetic);
  * backward dx: bit-identical (same u, t1 and dx GEMM order); dgamma / dbeta: the same sums over a different
    pixel partition (other blocks, other tile order), equal to fp32 summation-order noise;
and both against the fp32 oracle of layers/gdn.py:77-92 on the same bf16 operands.
Ragged pixel counts (past the 16-pixel wave tile and the 64-pixel step) and row strides > C are covered (the lane
kernels are taken from 32768 pixels up; below, both settings run the LDS-tile kernels)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

BETA_MIN, OFF = 1e-6, 2 ** -18


def _setup(C, seed, dev):
    from compressai import _native
    from compressai._ops import _p

    g = torch.Generator().manual_seed(seed)
    ped = OFF ** 2
    beta_raw = torch.sqrt(torch.ones(C) + ped) + 0.1 * torch.rand(C, generator=g)
    gamma_raw = torch.sqrt(0.1 * torch.eye(C) + ped) + 0.02 * torch.rand(C, C, generator=g)
    br, gr = beta_raw.to(dev), gamma_raw.to(dev)
    beta = torch.empty(C, device=dev)
    gop = torch.empty(2 * C * C, dtype=torch.bfloat16, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _native.lib.cai_gdn_reparam(_p(br), _p(gr), C, BETA_MIN, OFF, _native.BF16, _p(beta), _p(gop), st)
    return br, gr, beta, gop


def _with_lane(on, fn):
    old = os.environ.get("CAI_GDN_LANE")
    os.environ["CAI_GDN_LANE"] = "1" if on else "0"
    try:
        return fn()
    finally:
        if old is None:
            del os.environ["CAI_GDN_LANE"]
        else:
            os.environ["CAI_GDN_LANE"] = old


def _operand(npix, C, ld, seed, dev, scale=1.0):
    t = torch.zeros(npix, ld, dtype=torch.bfloat16, device=dev)
    t[:, :C] = (scale * torch.randn(npix, C, generator=torch.Generator().manual_seed(seed))).to(dev, torch.bfloat16)
    return t


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("C", [64, 128, 192])
@pytest.mark.parametrize("npix,ld_pad", [(32768, 0), (40000, 0), (65549, 32)])
def test_gdn_fwd_lane_bit_identical(cuda, C, inverse, npix, ld_pad):
    from compressai import _native
    from compressai._ops import _p

    lib = _native.lib
    br, gr, beta, gop = _setup(C, 1, cuda)
    ld = C + ld_pad
    x = _operand(npix, C, ld, 2, cuda)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for on in (True, False):
        y = torch.full((npix, ld), 7.0, dtype=torch.bfloat16, device=cuda)
        rc = _with_lane(on, lambda: lib.cai_gdn_fwd(_native.BF16, _p(x), ld, npix, C, _p(gop), _p(beta), int(inverse),
                                                    _p(y), ld, st))
        assert rc == 0
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][:, :C], outs[1][:, :C])
    assert bool((outs[0][:, C:] == 7.0).all())          # nothing written past C in a strided row
    # fp32 reference on the same bf16 operands: y = x * rsqrt(beta + gamma x^2) (or * sqrt)
    xs = x[:, :C].float()
    gam = gop[: C * C].float().view(C, C)
    norm = (xs.to(torch.bfloat16).float() ** 2).to(torch.bfloat16).float() @ gam.t() + beta
    yr = xs * (torch.sqrt(norm) if inverse else torch.rsqrt(norm))
    err = (outs[0][:, :C].float() - yr).abs().max().item() / yr.abs().max().item()
    assert err < 1e-2


def _backward(lib, native, p, x, dy, ld, npix, C, gop, beta, br, gr, inverse, dev):
    st = torch.cuda.current_stream().cuda_stream
    dx = torch.full((npix, ld), 7.0, dtype=torch.bfloat16, device=dev)
    dbr, dgr = torch.empty(C, device=dev), torch.empty(C, C, device=dev)
    nb = lib.cai_gdn_backward_workspace_bytes(npix, C, native.BF16)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    rc = lib.cai_gdn_backward(native.BF16, p(x), ld, p(dy), ld, npix, C, p(gop), p(beta), int(inverse), p(dx), ld,
                              p(br), p(gr), BETA_MIN, OFF, p(dbr), p(dgr), 0, p(ws), nb, st)
    assert rc == 0
    return dx, dbr, dgr


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("npix,ld_pad", [(32768, 0), (40009, 0), (65549, 32), (262144, 0)])
def test_gdn_bwd_lane_matches_fused(cuda, C, inverse, npix, ld_pad):
    from compressai import _native
    from compressai._ops import _p

    lib = _native.lib
    br, gr, beta, gop = _setup(C, 3, cuda)
    ld = C + ld_pad
    x = _operand(npix, C, ld, 4, cuda)
    dy = _operand(npix, C, ld, 5, cuda, 0.1)
    lane = _with_lane(True, lambda: _backward(lib, _native, _p, x, dy, ld, npix, C, gop, beta, br, gr, inverse, cuda))
    old = _with_lane(False, lambda: _backward(lib, _native, _p, x, dy, ld, npix, C, gop, beta, br, gr, inverse, cuda))
    again = _with_lane(True, lambda: _backward(lib, _native, _p, x, dy, ld, npix, C, gop, beta, br, gr, inverse, cuda))
    torch.cuda.synchronize()
    assert torch.equal(lane[0][:, :C], old[0][:, :C])                  # dx: bit-identical
    assert bool((lane[0][:, C:] == 7.0).all())
    for a, b in zip(lane[1:], again[1:]):                              # deterministic run to run
        assert torch.equal(a, b)
    for a, b in zip(lane[1:], old[1:]):                                # dbeta_raw, dgamma_raw: other partition
        scale = b.abs().max().item()
        assert (a - b).abs().max().item() <= 1e-4 * scale + 1e-30
    # the parameter gradients against fp64 sums over the same bf16 operands
    xs = x[:, :C].double()
    q = (xs.float() ** 2).to(torch.bfloat16).double()
    gam = gop[: C * C].double().view(C, C)
    norm = q @ gam.t() + beta.double()
    gs = dy[:, :C].double()
    u = (0.5 * gs * xs / torch.sqrt(norm)) if inverse else (-0.5 * gs * xs * norm ** -1.5)
    dgamma = u.t() @ q
    dbeta = u.sum(0)
    bb, gb = np.sqrt(BETA_MIN + OFF ** 2), OFF
    d_g = 2 * torch.clamp(gr.double(), min=gb) * dgamma
    d_b = 2 * torch.clamp(br.double(), min=bb) * dbeta
    assert (lane[2].double() - d_g).abs().max().item() < 2e-2 * d_g.abs().max().item()
    assert (lane[1].double() - d_b).abs().max().item() < 1e-3 * d_b.abs().max().item()
