"""The evaluation harness (python -m compressai.utils.eval_model) on the GPU vs the CPU oracle.

North-star bar: PSNR and bpp of the entropy-estimation eval within 1e-4 (relative) of the
reference arithmetic on identical inputs -- here the oracle's eval-mode forward with the same
weights, the same pad-to-64 / crop (eval_model/__main__t.py:149-211) and the same metric
formulas.  Real coding: the rate from the rANS strings tracks the estimate.
"""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import cai_oracle as O

pytestmark = pytest.mark.gpu


def _write_images(tmp_path, shapes, seed=0):
    from PIL import Image

    rng = np.random.default_rng(seed)
    d = tmp_path / "imgs"
    d.mkdir()
    paths = []
    for i, (h, w) in enumerate(shapes):
        # smooth-ish content: low-frequency pattern + noise (compressible, not constant)
        yy, xx = np.mgrid[0:h, 0:w]
        base = np.stack([np.sin(xx / (7 + c) + yy / (11 + 2 * c)) for c in range(3)], -1) * 0.35 + 0.5
        img = np.clip(base + rng.normal(0, 0.05, base.shape), 0, 1)
        p = d / f"img{i}.png"
        Image.fromarray((img * 255).round().astype(np.uint8)).save(p)
        paths.append(str(p))
    return str(d), paths


def _oracle_estimate(ref, path):
    from compressai.utils.eval_model.__main__ import _crop, _pad, read_image

    x = read_image(path).unsqueeze(0)
    xp, pads = _pad(x)
    with torch.no_grad():
        out = ref(xp)
    n = x.size(2) * x.size(3)
    bpp = sum((torch.log(l).sum() / (-math.log(2) * n)) for l in out["likelihoods"].values()).item()
    mse = F.mse_loss(x, _crop(out["x_hat"], pads)).item()
    return {"psnr": -10 * math.log10(mse), "bpp": bpp}


def test_entropy_estimation_matches_oracle(cuda, tmp_path):
    from compressai.utils.eval_model.__main__ import main

    torch.manual_seed(0)
    ref = O.ScaleHyperprior(32, 48).eval()
    ckpt = tmp_path / "ckpt.pth"
    torch.save({"state_dict": ref.state_dict()}, ckpt)
    d, paths = _write_images(tmp_path, [(80, 96), (64, 64), (130, 70)])
    out = main(["checkpoint", d, "-a", "bmshj2018-hyperprior", "-p", str(ckpt), "--entropy-estimation", "--cuda"])
    want = {"psnr": 0.0, "bpp": 0.0}
    for p in paths:
        r = _oracle_estimate(ref, p)
        for k in want:
            want[k] += r[k] / len(paths)
    for k, v in want.items():
        got = out["results"][k][0]
        assert abs(got - v) <= 1e-4 * abs(v), (k, got, v)


def test_real_coding_rate_tracks_estimate(cuda, tmp_path):
    from compressai.utils.eval_model.__main__ import main

    torch.manual_seed(1)
    ref = O.MeanScaleHyperprior(32, 48).eval()
    ckpt = tmp_path / "ckpt.pth"
    torch.save(ref.state_dict(), ckpt)
    d, _ = _write_images(tmp_path, [(192, 192), (176, 240)], seed=1)
    est = main(["checkpoint", d, "-a", "mbt2018-mean", "-p", str(ckpt), "--entropy-estimation", "--cuda"])
    real = main(["checkpoint", d, "-a", "mbt2018-mean", "-p", str(ckpt), "--cuda"])
    r, e = real["results"], est["results"]
    assert math.isfinite(r["psnr"][0]) and r["encoding_time"][0] > 0
    # strings carry a few bytes of rANS state per image and model: 0.9x .. 1.1x + overhead
    assert 0.9 * e["bpp"][0] <= r["bpp"][0] <= 1.1 * e["bpp"][0] + 0.05, (r["bpp"], e["bpp"])
    assert 0.0 < r["ms-ssim"][0] <= 1.0


def test_paired_eval_real_coding(cuda, tmp_path):
    """Paired (IR master + RGB guide) evaluation, __main__rgbt.py:99-178: real coding's rate tracks the
    entropy estimate plus the 64 beta + 64 gamma fp32 side values (:142); PSNR of real coding equals the
    estimate's within quantization-of-means noise."""
    from PIL import Image

    from compressai.models import Guided_compresser, Master_compresser
    from compressai.utils.eval_model.__main__ import main

    torch.manual_seed(2)
    m, g = Master_compresser(width=64, height=64, channel=1), Guided_compresser(channel=3)
    torch.save(m.state_dict(), tmp_path / "m.pth")
    torch.save(g.state_dict(), tmp_path / "g.pth")
    _, rgb_paths = _write_images(tmp_path, [(128, 128), (128, 128)], seed=3)
    ird = tmp_path / "ir"
    ird.mkdir()
    for i, p in enumerate(rgb_paths):
        Image.open(p).convert("L").resize((64, 64)).save(ird / f"ir{i}.png")
    args = ["checkpoint", str(ird), "-a", "Master_compresser", "-p", str(tmp_path / "m.pth"), "-ch", "1",
            "--guided-dataset", str(tmp_path / "imgs"), "--guided-checkpoint", str(tmp_path / "g.pth"), "--cuda"]
    est = main(args + ["--entropy-estimation"])["results"]
    with pytest.warns(UserWarning):
        real = main(args)["results"]
    side = 64 * 2 * 4 * 8 / (64 * 64)
    assert 0.9 * est["bpp"][0] + side <= real["bpp"][0] <= 1.1 * est["bpp"][0] + side + 0.05, (real, est)
    assert math.isfinite(real["psnr"][0]) and real["encoding_time"][0] > 0
