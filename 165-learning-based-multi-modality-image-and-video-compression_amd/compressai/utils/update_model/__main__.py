"""Update the CDF buffers of a trained checkpoint (reference: compressai/utils/update_model/__main__.py).

After training, ``net.update(force=True)`` builds the entropy coder's tables (quantized CDFs, offsets, CDF
lengths: EntropyBottleneck / GaussianConditional ``update``, libcai_coder.so) and the model is re-saved as
``<name>-<sha256 prefix><ext>`` so it loads like a zoo checkpoint.  The CLI is the reference's:

  python -m compressai.utils.update_model CKPT [-a ARCH] [-n NAME] [-d DIR] [-c CHANNEL] [--no-update]

ARCH: a zoo name (``bmshj2018-hyperprior``, ``cheng2020-attn``, ...), one of the class aliases
(``factorized-prior``, ``scale-hyperprior``, ``mean-scale-hyperprior``, ``jarhp``) or ``Guided_compresser`` /
``Master_compresser`` (the paired codec, width 512 x height 640 as the reference builds it).  Differences from
the reference: checkpoints are read with ``torch.load(weights_only=True)`` (tensors only, nothing executed);
the video model (``ssf2020``) and the depth-map variants (``cheng2020-attn_R`` / ``_D``) are not part of this
build and are refused with a ValueError.
"""
from __future__ import annotations

import argparse
import hashlib
import sys
from pathlib import Path
from typing import Dict

import torch

from compressai.models import (FactorizedPrior, Guided_compresser, JointAutoregressiveHierarchicalPriors,
                               Master_compresser, MeanScaleHyperprior, ScaleHyperprior)
from compressai.zoo import load_state_dict
from compressai.zoo.image import model_architectures as zoo_models

models = {
    "factorized-prior": FactorizedPrior,
    "jarhp": JointAutoregressiveHierarchicalPriors,
    "mean-scale-hyperprior": MeanScaleHyperprior,
    "scale-hyperprior": ScaleHyperprior,
}
models.update(zoo_models)
_NOT_BUILT = ("ssf2020", "cheng2020-attn_R", "cheng2020-attn_D")


def sha256_file(filepath: Path, len_hash_prefix: int = 8) -> str:
    """update_model/__main__.py:60-71."""
    sha256 = hashlib.sha256()
    with filepath.open("rb") as f:
        for buf in iter(lambda: f.read(8192), b""):
            sha256.update(buf)
    return sha256.hexdigest()[:len_hash_prefix]


def load_checkpoint(filepath: Path) -> Dict[str, torch.Tensor]:
    """update_model/__main__.py:74-86: the state dict under "network" / "state_dict" or the file itself,
    with the zoo's key migration (DataParallel prefixes, old entropy-bottleneck names)."""
    checkpoint = torch.load(filepath, map_location="cpu", weights_only=True)
    if "network" in checkpoint:
        state_dict = checkpoint["network"]
    elif "state_dict" in checkpoint:
        state_dict = checkpoint["state_dict"]
    else:
        state_dict = checkpoint
    return load_state_dict(state_dict)


description = """
Export a trained model to a new checkpoint with an updated CDFs parameters and a
hash prefix, so that it can be loaded later via `load_state_dict_from_url`.
""".strip()


def setup_args():
    parser = argparse.ArgumentParser(description=description)
    parser.add_argument("filepath", type=str, help="Path to the checkpoint model to be exported.")
    parser.add_argument("-n", "--name", type=str, help="Exported model name.")
    parser.add_argument("-d", "--dir", type=str, help="Exported model directory.")
    parser.add_argument("-c", "--channel", type=int, default=3, help="image channel")
    parser.add_argument("--no-update", action="store_true", default=False,
                        help="Do not update the model CDFs parameters.")
    parser.add_argument("-a", "--architecture", default="scale-hyperprior",
                        help="Set model architecture (default: %(default)s).")
    return parser


def build(architecture: str, state_dict, channel: int):
    """The model of `architecture` carrying `state_dict` (update_model/__main__.py:136-176)."""
    if architecture in _NOT_BUILT:
        raise ValueError(f'architecture "{architecture}" is not part of this build')
    if architecture == "Guided_compresser":
        net = Guided_compresser(channel=channel)
        net.load_state_dict(state_dict)
        return net
    if architecture == "Master_compresser":
        net = Master_compresser(width=512, height=640, channel=channel)
        net.load_state_dict(state_dict)
        return net
    if architecture not in models:
        raise ValueError(f'unknown architecture "{architecture}" (known: {", ".join(sorted(models))})')
    return models[architecture].from_state_dict(state_dict, channel=channel)


def main(argv):
    args = setup_args().parse_args(argv)
    filepath = Path(args.filepath).resolve()
    if not filepath.is_file():
        raise RuntimeError(f'"{filepath}" is not a valid file.')
    net = build(args.architecture, load_checkpoint(filepath), args.channel)
    if not args.no_update:
        net.update(force=True)
    state_dict = net.state_dict()

    if not args.name:
        filename = filepath
        while filename.suffixes:
            filename = Path(filename.stem)
    else:
        filename = args.name
    ext = "".join(filepath.suffixes)
    output_dir = Path(args.dir) if args.dir is not None else Path.cwd()
    output_dir.mkdir(exist_ok=True)
    # the reference saves `<name>_update.<ext>` then renames it to `<name>-<hash><ext>` (in the working
    # directory); here both live in the output directory
    tmp = output_dir / f"{Path(filename).name}_update{ext}"
    torch.save(state_dict, tmp)
    hash_prefix = sha256_file(tmp)
    out = output_dir / f"{Path(filename).name}-{hash_prefix}{ext}"
    tmp.rename(out)
    print(out)
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
