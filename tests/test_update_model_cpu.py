"""compressai.utils.update_model (reference: compressai/utils/update_model/__main__.py): a trained checkpoint is
rebuilt, its CDF tables updated (net.update(force=True): libcai_coder.so, host C++) and re-saved under a
sha256-prefixed name; the result loads into a fresh model with populated entropy-coder buffers equal to a
direct update().  CPU only (model construction, update() and the coder run on the host)."""
import hashlib

import pytest
import torch


def _ckpt(tmp_path, net, key):
    p = tmp_path / "model.pth.tar"
    torch.save({key: net.state_dict()} if key else net.state_dict(), p)
    return p


@pytest.mark.parametrize("arch,key", [("scale-hyperprior", "state_dict"), ("bmshj2018-factorized", "network"),
                                      ("mbt2018-mean", None)])
def test_update_model_writes_hashed_checkpoint(tmp_path, arch, key):
    from compressai.models import FactorizedPrior, MeanScaleHyperprior, ScaleHyperprior
    from compressai.utils.update_model.__main__ import main

    cls = {"scale-hyperprior": ScaleHyperprior, "bmshj2018-factorized": FactorizedPrior,
           "mbt2018-mean": MeanScaleHyperprior}[arch]
    torch.manual_seed(0)
    net = cls(16, 24)
    src = _ckpt(tmp_path, net, key)
    out = main([str(src), "-a", arch, "-d", str(tmp_path / "out")])
    assert out.name.startswith("model-") and out.name.endswith(".pth.tar")
    digest = hashlib.sha256(out.read_bytes()).hexdigest()[:8]
    assert out.name == f"model-{digest}.pth.tar"
    sd = torch.load(out, weights_only=True)
    assert sd["entropy_bottleneck._quantized_cdf"].numel() > 0
    ref = cls(16, 24)
    ref.load_state_dict(net.state_dict())
    ref.update(force=True)
    for k in ("entropy_bottleneck._quantized_cdf", "entropy_bottleneck._offset", "entropy_bottleneck._cdf_length"):
        assert torch.equal(sd[k], ref.state_dict()[k]), k
    if arch != "bmshj2018-factorized":
        assert torch.equal(sd["gaussian_conditional._quantized_cdf"], ref.gaussian_conditional._quantized_cdf)
    fresh = cls.from_state_dict(sd)
    assert torch.equal(fresh.entropy_bottleneck._quantized_cdf, ref.entropy_bottleneck._quantized_cdf)


def test_update_model_no_update_and_refusals(tmp_path):
    from compressai.models import ScaleHyperprior
    from compressai.utils.update_model.__main__ import main

    torch.manual_seed(1)
    src = _ckpt(tmp_path, ScaleHyperprior(16, 24), "state_dict")
    out = main([str(src), "--no-update", "-n", "plain", "-d", str(tmp_path)])
    assert out.name.startswith("plain-")
    assert torch.load(out, weights_only=True)["entropy_bottleneck._quantized_cdf"].numel() == 0
    with pytest.raises(ValueError):
        main([str(src), "-a", "ssf2020", "-d", str(tmp_path)])
    with pytest.raises(RuntimeError):
        main([str(tmp_path / "missing.pth"), "-d", str(tmp_path)])
