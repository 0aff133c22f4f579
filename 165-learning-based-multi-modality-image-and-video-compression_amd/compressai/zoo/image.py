"""Model registry (reference: compressai/zoo/image.py:52-411).

(name, quality) -> (class, N, M).  Pretrained weights are S3 downloads in the
reference; this build has no network, so ``pretrained=True`` raises.
"""
from ..models import (FactorizedPrior, JointAutoregressiveHierarchicalPriors, MeanScaleHyperprior,
                      ScaleHyperprior)

__all__ = ["bmshj2018_factorized", "bmshj2018_hyperprior", "mbt2018", "mbt2018_mean"]

model_architectures = {
    "bmshj2018-factorized": FactorizedPrior,
    "bmshj2018-hyperprior": ScaleHyperprior,
    "mbt2018-mean": MeanScaleHyperprior,
    "mbt2018": JointAutoregressiveHierarchicalPriors,
}

cfgs = {
    "bmshj2018-factorized": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "bmshj2018-hyperprior": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "mbt2018-mean": {q: ((128, 192) if q <= 4 else (192, 320)) for q in range(1, 9)},
    "mbt2018": {q: ((192, 192) if q <= 4 else (192, 320)) for q in range(1, 9)},
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
