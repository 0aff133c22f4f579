"""Evaluation harness pieces that run without a GPU: metrics, padding, CLI parsing."""
import math

import pytest
import torch


def test_psnr_matches_formula():
    from compressai.utils.metrics import psnr

    a = torch.rand(1, 3, 16, 16, generator=torch.Generator().manual_seed(0))
    b = a + 0.01
    assert abs(psnr(a, b) - (-10 * math.log10(1e-4))) < 1e-3


def test_ms_ssim_properties():
    from compressai.utils.metrics import ms_ssim

    g = torch.Generator().manual_seed(1)
    x = torch.rand(1, 3, 192, 176, generator=g)
    assert abs(ms_ssim(x, x).item() - 1.0) < 1e-6
    n1 = ms_ssim(x, (x + 0.05 * torch.randn(x.shape, generator=g)).clamp(0, 1)).item()
    n2 = ms_ssim(x, (x + 0.2 * torch.randn(x.shape, generator=g)).clamp(0, 1)).item()
    assert 1.0 > n1 > n2 > 0.0
    with pytest.raises(ValueError):
        ms_ssim(torch.rand(1, 1, 100, 100), torch.rand(1, 1, 100, 100))   # too small for 5 scales


def test_pad_crop_round_trip():
    from compressai.utils.eval_model.__main__ import _crop, _pad

    x = torch.rand(1, 3, 70, 131)
    xp, pads = _pad(x)
    assert xp.shape[-2:] == (128, 192) and pads == (30, 31, 29, 29)
    assert torch.equal(_crop(xp, pads), x)


def test_cli_parsing():
    from compressai.utils.eval_model.__main__ import setup_args

    a = setup_args().parse_args(["checkpoint", "/data", "-a", "bmshj2018-hyperprior", "-p", "x.pth", "--entropy-estimation"])
    assert a.source == "checkpoint" and a.paths == ["x.pth"] and a.entropy_estimation and a.entropy_coder == "ans"


def test_rename_keys():
    from compressai.zoo import load_state_dict

    sd = load_state_dict({"module.entropy_bottleneck._biases.2": 0, "g_a.0.downsample.weight": 1, "h_a.0.weight": 2})
    assert sd == {"entropy_bottleneck._bias2": 0, "g_a.0.skip.weight": 1, "h_a.0.weight": 2}
