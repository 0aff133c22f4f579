"""state_dict key migration (reference: compressai/zoo/pretrained.py:35-64).

Checkpoints written by the reference (DataParallel ``module.`` prefixes, the
old ``downsample`` / ParameterList names) load into this build's modules,
whose state_dict keys are the reference's.
"""
from typing import Dict

from torch import Tensor

__all__ = ["rename_key", "load_pretrained"]


def rename_key(key: str) -> str:
    if key.startswith("module."):
        key = key[7:]
    if ".downsample." in key:
        return key.replace("downsample", "skip")
    if key.startswith("entropy_bottleneck."):
        for old, new in (("_biases.", "_bias"), ("_matrices.", "_matrix"), ("_factors.", "_factor")):
            if key.startswith("entropy_bottleneck." + old):
                return f"entropy_bottleneck.{new}{key[-1]}"
    return key


def load_pretrained(state_dict: Dict[str, Tensor]) -> Dict[str, Tensor]:
    return {rename_key(k): v for k, v in state_dict.items()}
