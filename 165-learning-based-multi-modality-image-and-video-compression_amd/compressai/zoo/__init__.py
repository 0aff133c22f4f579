"""Model zoo (reference: compressai/zoo/__init__.py:30-56)."""
from .pretrained import load_pretrained
from .pretrained import load_pretrained as load_state_dict
from .image import (bmshj2018_factorized, bmshj2018_hyperprior, cfgs, cheng2020_anchor, cheng2020_attn, mbt2018,
                    mbt2018_mean, model_architectures)

image_models = {
    "bmshj2018-factorized": bmshj2018_factorized,
    "bmshj2018-hyperprior": bmshj2018_hyperprior,
    "mbt2018-mean": mbt2018_mean,
    "mbt2018": mbt2018,
    "cheng2020-anchor": cheng2020_anchor,
    "cheng2020-attn": cheng2020_attn,
}

models = dict(image_models)

__all__ = ["image_models", "models", "cfgs", "model_architectures", "load_state_dict", "load_pretrained"]
