"""Bitstream path on the GPU models: update() CDF tables, compress / decompress round trips.

Reference behaviour pinned here:
  * EntropyBottleneck compress -> decompress == round(x) for 2-D .. 5-D inputs
    (tests/test_entropy_models.py:258-283);
  * update() tables within 2 of an independent computation (the reference's own
    tolerance, tests/test_entropy_models.py:382-398) -- here the oracle's CPU
    restatement of update() (entropy_models.py:396-441, 655-678) quantized by the
    pure-Python pmf_to_quantized_cdf;
  * decompress(compress(x)) reproduces the eval-mode forward's reconstruction
    (the decoder sees exactly the encoder's y_hat), and the real rate stays near
    the estimated one (eval_model/__main__t.py:137-138 vs :195-200).
"""
import math

import numpy as np
import pytest
import torch

import cai_coder_oracle as OC
import cai_oracle as O

pytestmark = pytest.mark.gpu


def _oracle_eb_tables(eb_ref):
    """CPU restatement of EntropyBottleneck.update (entropy_models.py:396-441)."""
    with torch.no_grad():
        q = eb_ref.quantiles
        medians = q[:, 0, 1]
        minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
        maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
        pmf_start = medians - minima
        pmf_length = maxima + minima + 1
        L = int(pmf_length.max())
        samples = torch.arange(L)[None, :] + pmf_start[:, None, None]
        lower = eb_ref._logits_cumulative(samples - 0.5, stop_gradient=True)
        upper = eb_ref._logits_cumulative(samples + 0.5, stop_gradient=True)
        sign = -torch.sign(lower + upper)
        pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
        tail = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    cdf = np.zeros((len(pmf_length), L + 2), dtype=np.int64)
    for i, n in enumerate(pmf_length.tolist()):
        c = OC.pmf_to_quantized_cdf(pmf[i, :n].tolist() + [float(tail[i, 0])], 16)
        cdf[i, :len(c)] = c
    return cdf, (-minima).numpy(), (pmf_length + 2).numpy()


@pytest.mark.parametrize("dims", [0, 1, 2, 3])
def test_eb_compression_nd(cuda, dims):
    from compressai.entropy_models import EntropyBottleneck

    torch.manual_seed(0)
    eb = EntropyBottleneck(128).to(cuda)
    eb.update()
    x = torch.rand(2, 128, *([4] * dims), generator=torch.Generator().manual_seed(dims)).to(cuda) * 6 - 3
    s = eb.compress(x)
    assert len(s) == 2 and all(isinstance(b, bytes) for b in s)
    x2 = eb.decompress(s, x.size()[2:])
    assert torch.equal(torch.round(x), x2)


def test_eb_tables_match_oracle(cuda):
    from compressai.entropy_models import EntropyBottleneck

    torch.manual_seed(1)
    ref = O.EntropyBottleneck(64)
    with torch.no_grad():
        ref.quantiles.copy_(torch.tensor([-4.3, 0.2, 5.1]).repeat(64, 1, 1) + torch.randn(64, 1, 3) * 0.5)
    eb = EntropyBottleneck(64)
    eb.load_state_dict(ref.state_dict(), strict=False)
    eb = eb.to(cuda)
    assert eb.update(force=True)
    assert not eb.update()
    cdf, off, length = _oracle_eb_tables(ref)
    assert np.array_equal(eb._offset.cpu().numpy(), off)
    assert np.array_equal(eb._cdf_length.cpu().numpy(), length)
    assert np.abs(eb._quantized_cdf.cpu().numpy().astype(np.int64) - cdf).max() <= 2


def test_gc_tables_match_oracle(cuda):
    from compressai.entropy_models import GaussianConditional
    from compressai.models import get_scale_table

    gc = GaussianConditional(None).to(cuda)
    table = get_scale_table()
    assert gc.update_scale_table(table)
    assert not gc.update_scale_table(table)
    # entropy_models.py:655-678 on the CPU, quantized by the oracle
    mult = 6.109410204869  # -norm.ppf(1e-9 / 2)
    st = table.float()
    center = torch.ceil(st * mult).int()
    assert torch.equal(gc._offset.cpu(), -center)
    length = 2 * center + 1
    assert torch.equal(gc._cdf_length.cpu(), length + 2)
    L = int(length.max())
    samples = torch.abs(torch.arange(L).int() - center[:, None]).float()
    upper = 0.5 * torch.erfc(-(2 ** -0.5) * (0.5 - samples) / st[:, None])
    lower = 0.5 * torch.erfc(-(2 ** -0.5) * (-0.5 - samples) / st[:, None])
    pmf = upper - lower
    tab = gc._quantized_cdf.cpu().numpy()
    for i in (0, 1, 17, 40, 63):
        n = int(length[i])
        c = OC.pmf_to_quantized_cdf(pmf[i, :n].tolist() + [float(2 * lower[i, 0])], 16)
        assert np.abs(tab[i, :len(c)].astype(np.int64) - np.array(c)).max() <= 2


def _bits(strings):
    return sum(len(b) for s in strings for b in (s if isinstance(s, list) else [s])) * 8


@pytest.mark.parametrize("name", ["FactorizedPrior", "ScaleHyperprior", "MeanScaleHyperprior"])
def test_model_round_trip(cuda, name):
    import compressai.models as M

    torch.manual_seed(3)
    net = getattr(M, name)(32, 48).to(cuda).eval()
    net.update()
    x = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(4)).to(cuda)
    with torch.no_grad():
        out = net(x)
    enc = net.compress(x)
    dec = net.decompress(enc["strings"], enc["shape"])
    # the decoder rebuilds exactly the eval forward's y_hat
    assert (dec["x_hat"] - out["x_hat"].clamp(0, 1)).abs().max().item() < 1e-5
    est = sum(torch.log(l).sum().item() for l in out["likelihoods"].values()) / -math.log(2)
    real = _bits(enc["strings"])
    nstr = sum(len(s) for s in enc["strings"])
    assert 0.9 * est <= real <= 1.1 * est + 64 * nstr, (real, est)


def test_autoregressive_round_trip(cuda):
    """JointAutoregressiveHierarchicalPriors: serial context coding; the decoder's y_hat
    equals the encoder's (google.py:565-692)."""
    import torch.nn.functional as F

    from compressai.models import JointAutoregressiveHierarchicalPriors

    torch.manual_seed(5)
    net = JointAutoregressiveHierarchicalPriors(32, 48).to(cuda).eval()
    net.update()
    x = torch.rand(1, 3, 64, 64, generator=torch.Generator().manual_seed(6)).to(cuda)
    with pytest.warns(UserWarning):
        enc = net.compress(x)
    with pytest.warns(UserWarning):
        dec = net.decompress(enc["strings"], enc["shape"])
    assert dec["x_hat"].shape == x.shape and torch.isfinite(dec["x_hat"]).all()
    with pytest.warns(UserWarning):
        enc2 = net.compress(x)
    assert enc2["strings"] == enc["strings"]          # deterministic kernels
    # encoder-side y_hat, rebuilt with the same loop, vs the decoder's
    from compressai._prepack import prepacked_forward

    with torch.no_grad(), prepacked_forward(net):
        y = net.g_a(x)
        z_hat = net.entropy_bottleneck.decompress(enc["strings"][1], enc["shape"])
        params = net.h_s(z_hat)
        y_enc = F.pad(y.float(), (2, 2, 2, 2))
        H, W = y.shape[2], y.shape[3]
        s = net._compress_ar(y_enc, params, H, W, 5, 2)
        assert s == enc["strings"][0][0]
        y_dec = torch.zeros_like(y_enc)
        net._decompress_ar(s, y_dec, params, H, W, 5, 2)
    assert torch.equal(y_enc[:, :, 2:-2, 2:-2], y_dec[:, :, 2:-2, 2:-2])


def test_multimodal_round_trip(cuda):
    """Guided_compresser / Master_compresser compress -> decompress (master.py:953-1147, 1297-1464): the
    decoder rebuilds exactly the encoder-side reconstruction (same y_hat, same aligned guide)."""
    import torch.nn.functional as F

    from compressai._ops import CatFn, ChannelAffineFn
    from compressai._prepack import prepacked_forward
    from compressai.models import Guided_compresser, Master_compresser

    torch.manual_seed(7)
    g = Guided_compresser(channel=3).to(cuda).eval()
    m = Master_compresser(width=64, height=64, channel=1).to(cuda).eval()
    g.update()
    m.update()
    x = torch.rand(1, 1, 64, 64, generator=torch.Generator().manual_seed(8)).to(cuda)
    rgb = torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(9)).to(cuda)
    with pytest.warns(UserWarning):
        enc_g = g.compress(rgb)
    with pytest.warns(UserWarning):
        dec_g = g.decompress(enc_g["strings"], enc_g["shape"])
    assert dec_g["x_hat"].shape == rgb.shape and set(dec_g["hidden"]) == {"gs1", "gs2", "gs3"}
    enc_m = m.compress(x, dec_g["x_hat"])
    assert enc_m["gamma"].shape == (1, 64, 1, 1) and enc_m["beta"].shape == (1, 64, 1, 1)
    with pytest.warns(UserWarning):
        dec_m = m.decompress(enc_m, dec_g)
    # encoder-side reconstruction
    with torch.no_grad(), prepacked_forward(m):
        xf = m.fencoder1(x)
        ga, beta, gamma = m.ch_aligner(xf, m.fencoder2(dec_g["x_hat"]))
        y = m.g_a(CatFn.apply(xf, ga))
        z_hat = m.entropy_bottleneck.decompress(enc_m["strings"][1], enc_m["shape"])
        params = m.h_s(z_hat)
        y_enc = F.pad(y.float(), (2, 2, 2, 2))
        s = m._compress_ar(y_enc, params, y.shape[2], y.shape[3], 5, 2)
        assert s == enc_m["strings"][0][0]
        res = m.decoder(y_enc[:, :, 2:-2, 2:-2].contiguous(), dec_g["hidden"])
        ga2 = ChannelAffineFn.apply(m.fencoder2(dec_g["x_hat"]), gamma, beta)
        x_rec = m.fdecoder(CatFn.apply(res["x_feature_hat"], ga2)).clamp_(0, 1)
    assert torch.equal(dec_m["x_hat"], x_rec)


def test_codec_rgbt_file_round_trip(cuda, tmp_path):
    """codec_rgbt.py encode_image / decode_image through the container file: the Master stream decodes to the
    same image as the in-memory decompress; bpp is the file size over the master's pixels."""
    import warnings

    from compressai.models import Guided_compresser, Master_compresser
    from compressai.utils.codec_rgbt import decode_image, encode_image
    from compressai.zoo import bmshj2018_hyperprior

    torch.manual_seed(11)
    g = Guided_compresser(channel=3).to(cuda).eval()
    m = Master_compresser(width=64, height=64, channel=1).to(cuda).eval()
    g.update()
    m.update()
    x = torch.rand(1, 1, 64, 64, generator=torch.Generator().manual_seed(12)).to(cuda)
    rgb = torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(13)).to(cuda)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        path = tmp_path / "m.bin"
        r = encode_image(x, [g, m], str(path), "Master_compresser", "mse", 3, guided=rgb)
        assert r["bpp"] == path.stat().st_size * 8.0 / (64 * 64)
        hdr, x_hat = decode_image(str(path), [g, m], guided=rgb)
        assert hdr == ("Master_compresser", "mse", 3, (64, 64), 8)
        dec_g = g.decompress(*(lambda e: (e["strings"], e["shape"]))(g.compress(rgb)))
        ref = m.decompress(m.compress(x, dec_g["x_hat"]), dec_g)["x_hat"]
        assert torch.equal(x_hat, ref)

        net = bmshj2018_hyperprior(1, channel=3).to(cuda).eval()
        net.update()
        path = tmp_path / "h.bin"
        encode_image(rgb, net, str(path), "bmshj2018-hyperprior", "mse", 1)
        hdr, x_hat = decode_image(str(path), net)
        enc = net.compress(rgb)
        assert hdr.model == "bmshj2018-hyperprior"
        assert torch.equal(x_hat, net.decompress(enc["strings"], enc["shape"])["x_hat"])
