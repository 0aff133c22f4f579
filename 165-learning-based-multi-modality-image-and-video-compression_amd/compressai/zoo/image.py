"""Model registry (reference: compressai/zoo/image.py:52-411).

(name, quality) -> (class, N, M).  Pretrained weights are S3 downloads in the
reference; this build has no network, so ``pretrained=True`` raises.
"""
from ..models import (Cheng2020Anchor, Cheng2020Attention, FactorizedPrior, JointAutoregressiveHierarchicalPriors,
                      MeanScaleHyperprior, ScaleHyperprior)

__all__ = ["bmshj2018_factorized", "bmshj2018_hyperprior", "mbt2018", "mbt2018_mean", "cheng2020_anchor",
           "cheng2020_attn"]

model_architectures = {
    "bmshj2018-factorized": FactorizedPrior,
    "bmshj2018-hyperprior": ScaleHyperprior,
    "mbt2018-mean": MeanScaleHyperprior,
    "mbt2018": JointAutoregressiveHierarchicalPriors,
    "cheng2020-anchor": Cheng2020Anchor,
    "cheng2020-attn": Cheng2020Attention,
}

cfgs = {
    "bmshj2018-factorized": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "bmshj2018-hyperprior": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "mbt2018-mean": {q: ((128, 192) if q <= 4 else (192, 320)) for q in range(1, 9)},
    "mbt2018": {q: ((192, 192) if q <= 4 else (192, 320)) for q in range(1, 9)},
    "cheng2020-anchor": {q: ((128,) if q <= 3 else (192,)) for q in range(1, 7)},
    "cheng2020-attn": {q: ((128,) if q <= 3 else (192,)) for q in range(1, 7)},
}


def _load_model(architecture, metric, quality, pretrained=False, progress=True, channel=3, **kwargs):
    if architecture not in model_architectures:
        raise ValueError(f'Invalid architecture name "{architecture}"')
    if quality not in cfgs[architecture]:
        raise ValueError(f'Invalid quality value "{quality}"')
    if pretrained:
        raise RuntimeError("Pre-trained weights are remote downloads in the reference; not available offline")
    return model_architectures[architecture](*cfgs[architecture][quality], channel=channel, **kwargs)


def _check_metric(metric):
    if metric not in ("mse", "ms-ssim"):
        raise ValueError(f'Invalid metric "{metric}"')


def bmshj2018_factorized(quality, channel=3, metric="mse", pretrained=False, progress=True, **kwargs):
    _check_metric(metric)
    if quality < 1 or quality > 8:
        raise ValueError(f'Invalid quality "{quality}", should be between (1, 8)')
    return _load_model("bmshj2018-factorized", metric, quality, pretrained, progress, channel=channel, **kwargs)


def bmshj2018_hyperprior(quality, channel=3, metric="mse", pretrained=False, progress=True, **kwargs):
    _check_metric(metric)
    if quality < 1 or quality > 8:
        raise ValueError(f'Invalid quality "{quality}", should be between (1, 8)')
    return _load_model("bmshj2018-hyperprior", metric, quality, pretrained, progress, channel=channel, **kwargs)


def mbt2018_mean(quality, channel=3, metric="mse", pretrained=False, progress=True, **kwargs):
    _check_metric(metric)
    if quality < 1 or quality > 8:
        raise ValueError(f'Invalid quality "{quality}", should be between (1, 8)')
    return _load_model("mbt2018-mean", metric, quality, pretrained, progress, channel=channel, **kwargs)


def mbt2018(quality, channel=3, metric="mse", pretrained=False, progress=True, **kwargs):
    _check_metric(metric)
    if quality < 1 or quality > 8:
        raise ValueError(f'Invalid quality "{quality}", should be between (1, 8)')
    return _load_model("mbt2018", metric, quality, pretrained, progress, channel=channel, **kwargs)


def cheng2020_anchor(quality, channel=3, metric="mse", pretrained=False, progress=True, **kwargs):
    """zoo/image.py:368-388."""
    _check_metric(metric)
    if quality < 1 or quality > 6:
        raise ValueError(f'Invalid quality "{quality}", should be between (1, 6)')
    return _load_model("cheng2020-anchor", metric, quality, pretrained, progress, channel=channel, **kwargs)


def cheng2020_attn(quality, channel=3, metric="mse", pretrained=False, progress=True, **kwargs):
    """zoo/image.py:391-411."""
    _check_metric(metric)
    if quality < 1 or quality > 6:
        raise ValueError(f'Invalid quality "{quality}", should be between (1, 6)')
    return _load_model("cheng2020-attn", metric, quality, pretrained, progress, channel=channel, **kwargs)
