"""MI355X-native (gfx950) drop-in for the `compressai` training / entropy-estimation hot path.

Module paths, class names, constructor arguments and state_dict keys follow
the reference CompressAI 1.2.0.dev0 fork (/root/reference/CompressAI); the
forward/backward arithmetic runs in HIP kernels through libcai.so
(include/cai.h).  See DESIGN.md.
"""
from . import entropy_models, layers, models, ops, zoo  # noqa: F401
from ._native import available as native_available  # noqa: F401
from ._ops import set_fp16_autocast_policy  # noqa: F401

__version__ = "1.2.0.dev0+mi355x"

_entropy_coder = "ans"


def available_entropy_coders():
    return ["ans"]


def set_entropy_coder(entropy_coder):
    global _entropy_coder
    if entropy_coder not in available_entropy_coders():
        raise ValueError(f'Invalid entropy coder "{entropy_coder}", choose from ({", ".join(available_entropy_coders())}).')
    _entropy_coder = entropy_coder


def get_entropy_coder():
    return _entropy_coder
