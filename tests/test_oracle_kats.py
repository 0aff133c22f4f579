"""Pin the CPU oracle (oracle/cai_oracle.py) against the reference's own
known-answer tests, transcribed from /root/reference/CompressAI/tests (the
reference itself may not be imported here), plus an
independent check of the Gaussian likelihood against scipy.stats.norm.
"""
import math

import numpy as np
import pytest
import scipy.stats
import torch

import cai_oracle as O


# ---- tests/test_ops.py:37-101 ----------------------------------------------
def test_ste_round():
    x = torch.rand(24, requires_grad=True)
    y = O.ste_round(x)
    assert (y == torch.round(x)).all()
    y.backward(x)
    assert (x.grad == x).all()


def test_lower_bound_value_and_grad():
    x = torch.rand(16, requires_grad=True)
    bound = torch.rand(1)
    lb = O.LowerBound(bound)
    y = lb(x)
    assert (y == torch.max(x, bound)).all()
    y.backward(x)
    assert (x.grad == ((x >= bound) * x)).all()


def test_lower_bound_negative_grad_passes():
    # bound_ops.py:40-42: gradient passes when it pushes x upwards (grad < 0)
    x = torch.tensor([0.1, 0.9], requires_grad=True)
    y = O.LowerBound(0.5)(x)
    y.backward(torch.tensor([-1.0, -1.0]))
    assert torch.equal(x.grad, torch.tensor([-1.0, -1.0]))


def test_non_negative_parametrizer():
    p = O.NonNegativeParametrizer()
    x = torch.rand(1, 8, 8, 8) * 2 - 1
    r = p(x)
    assert r.shape == x.shape and r.min() >= 0
    xi = p.init(x)
    assert torch.allclose(xi, torch.sqrt(torch.max(x, x - x)), atol=2 ** -18)
    for _ in range(10):
        m = torch.rand(1)
        p = O.NonNegativeParametrizer(m.item())
        assert torch.allclose(p(torch.rand(1, 8, 8, 8) * 2 - 1).min(), m)


# ---- tests/test_layers.py:134-172 (GDN closed forms at init) -----------------
def test_gdn_closed_forms():
    x = torch.rand(1, 32, 16, 16, requires_grad=True)
    y = O.GDN(32)(x)
    y.backward(x)
    assert x.grad is not None and torch.allclose(x / torch.sqrt(1 + 0.1 * x ** 2), y)
    x = torch.rand(1, 32, 16, 16)
    assert torch.allclose(x * torch.sqrt(1 + 0.1 * x ** 2), O.GDN(32, inverse=True)(x))
    assert torch.allclose(x / (1 + 0.1 * torch.abs(x)), O.GDN1(32)(x))


# ---- tests/test_layers.py:45-128 (MaskedConv2d masks) ------------------------
def test_masked_conv_masks():
    c = O.MaskedConv2d(1, 3, 5, padding=2, mask_type="A")
    m = torch.ones(5, 5)
    m[2, 2:] = 0
    m[3:] = 0
    assert (c.mask[0, 0] == m).all()
    c = O.MaskedConv2d(1, 3, 5, padding=2, mask_type="B")
    m = torch.ones(5, 5)
    m[2, 3:] = 0
    m[3:] = 0
    assert (c.mask[0, 0] == m).all()
    with pytest.raises(ValueError):
        O.MaskedConv2d(1, 3, 5, mask_type="C")


# ---- tests/test_entropy_models.py:54-99 (quantize) ---------------------------
def test_quantize_semantics():
    em = O.EntropyModel()
    x = torch.rand(1, 3, 4, 4)
    with pytest.raises(ValueError):
        em.quantize(x, mode="toto")
    y = em.quantize(x, "noise")
    assert ((y - x) <= 0.5).all() and ((y - x) >= -0.5).all() and (y != torch.round(x)).any()
    assert (em.quantize(x, "symbols") == torch.round(x).int()).all()
    means = torch.rand(1, 3, 4, 4)
    assert (em.quantize(x, "dequantize", means) == torch.round(x - means) + means).all()
    xi = torch.randint(-32, 32, (1, 3, 4, 4))
    assert O.EntropyModel.dequantize(xi, means).type() == means.type()


def test_round_half_to_even():
    t = torch.tensor([0.5, 1.5, 2.5, -0.5, -1.5])
    assert torch.equal(O.EntropyModel().quantize(t[None], "symbols")[0], torch.tensor([0, 2, 2, 0, -2], dtype=torch.int32))


# ---- tests/test_entropy_models.py:163-221,312-363 (EB / GC forward) ----------
def test_eb_forward_semantics():
    eb = O.EntropyBottleneck(128)
    x = torch.rand(1, 128, 32, 32)
    y, lik = eb(x)
    assert y.shape == x.shape == lik.shape
    assert ((y - x) <= 0.5).all() and ((y - x) >= -0.5).all() and (y != torch.round(x)).any()
    eb.eval()
    for i in range(0, 6):
        x = torch.rand(1, 128, *([4] * i))
        y, lik = eb(x)
        assert y.shape == x.shape and lik.shape == x.shape
        assert (y == torch.round(x)).all()
    l = O.EntropyBottleneck(128).loss()
    assert l.dim() == 0 and l.numel() == 1


def test_gc_validation_and_semantics():
    for bad in (1, [], (), torch.rand(10), [2, 1], [0, 1, 2]):
        with pytest.raises(ValueError):
            O.GaussianConditional(bad)
    with pytest.raises(ValueError):
        O.GaussianConditional([], scale_bound=None)
    with pytest.raises(ValueError):
        O.GaussianConditional([], scale_bound=-0.1)
    gc = O.GaussianConditional(None)
    x, s, m = torch.rand(1, 128, 32, 32), torch.rand(1, 128, 32, 32), torch.rand(1, 128, 32, 32)
    y, lik = gc(x, s)
    assert ((y - x) <= 0.5).all() and ((y - x) >= -0.5).all()
    gc.eval()
    y, _ = gc(x, s)
    assert (y == torch.round(x)).all()
    y, _ = gc(x, s, m)
    assert (y == torch.round(x - m) + m).all()


def test_gc_likelihood_matches_scipy():
    """Independent pin: lik = Phi((1/2-|v|)/s) - Phi((-1/2-|v|)/s), s = max(scale, 0.11)."""
    gc = O.GaussianConditional(None).eval()
    rng = np.random.default_rng(0)
    v = rng.normal(0, 5, 4096).astype(np.float32)
    s = (rng.random(4096) * 6).astype(np.float32)
    s[:10] = 0.01
    _, lik = gc(torch.from_numpy(v)[None, :, None, None], torch.from_numpy(s)[None, :, None, None])
    vr = np.round(v).astype(np.float64)
    sb = np.maximum(s, 0.11).astype(np.float64)
    ref = scipy.stats.norm.cdf((0.5 - np.abs(vr)) / sb) - scipy.stats.norm.cdf((-0.5 - np.abs(vr)) / sb)
    ref = np.maximum(ref, 1e-9)
    got = lik[0, :, 0, 0].double().numpy()
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-7)


def test_eb_likelihood_is_a_pmf_at_init():
    """At init the EB density integrates to ~1 over the integer grid (a property of the
    reference construction: the chain is a monotone CDF logit)."""
    eb = O.EntropyBottleneck(4).eval()
    grid = torch.arange(-400, 401, dtype=torch.float32)
    x = grid[None, None, :].repeat(1, 4, 1)
    _, lik = eb(x)
    tot = lik.sum(-1)
    assert torch.allclose(tot, torch.ones_like(tot), atol=1e-3)


# ---- tests/test_models.py:53-58,77-181,242-259 -------------------------------
def test_compression_model_param_count():
    assert len(list(O.CompressionModel(32).parameters())) == 15
    with pytest.raises(NotImplementedError):
        O.CompressionModel(32)(torch.rand(1))


@pytest.mark.parametrize("cls,keys", [(O.FactorizedPrior, ("y",)), (O.ScaleHyperprior, ("y", "z")),
                                      (O.MeanScaleHyperprior, ("y", "z")),
                                      (O.JointAutoregressiveHierarchicalPriors, ("y", "z"))])
def test_model_shapes(cls, keys):
    torch.manual_seed(0)
    model = cls(128, 192)
    x = torch.rand(1, 3, 64, 64)
    out = model(x)
    assert out["x_hat"].shape == x.shape
    assert tuple(out["likelihoods"].keys()) == keys
    y = out["likelihoods"]["y"].shape
    assert y[1] == 192 and y[2] == 64 / 2 ** 4 and y[3] == 64 / 2 ** 4
    if "z" in keys:
        z = out["likelihoods"]["z"].shape
        assert z[1] == 128 and z[2] == 64 / 2 ** 6


def test_scale_table():
    t = O.get_scale_table()
    assert O.SCALES_MIN == 0.11 and O.SCALES_MAX == 256 and O.SCALES_LEVELS == 64
    assert t[0] == O.SCALES_MIN and t[-1] == O.SCALES_MAX and t.shape == (64,)
    t = O.get_scale_table(0.02, 1337, 32)
    assert t.shape == (32,) and abs(t[0].item() - 0.02) < 1e-6 and abs(t[-1].item() - 1337) < 1e-2


def test_parameter_counts_match_survey():
    """C2 5.08 M params, C3 7.03 M, C3' 14.13 M (incl. quantiles)."""
    n = lambda m: sum(p.numel() for p in m.parameters())
    assert abs(n(O.build("bmshj2018-hyperprior", 1)) / 1e6 - 5.08) < 0.01
    assert abs(n(O.build("mbt2018-mean", 1)) / 1e6 - 7.03) < 0.01
    assert abs(n(O.build("mbt2018", 1)) / 1e6 - 14.13) < 0.01
