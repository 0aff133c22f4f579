"""Evaluate a trained model on a directory of images.

Reference: compressai/utils/eval_model/__main__t.py (single modality) and
__main__rgbt.py (the paired RGB/IR codec).  Two modes, as there:

* ``--entropy-estimation``: pad to a multiple of 64 (__main__t.py:177-189),
  eval-mode ``forward()`` on the HIP kernels, bpp = sum(log likelihoods) /
  (-ln 2 * pixels) (:197-200), PSNR on the cropped reconstruction (:88-91,
  :202-204);
* real coding: ``compress()`` / ``decompress()`` (rANS strings from
  libcai_coder.so), bpp from the string lengths (:137-138), PSNR + MS-SSIM.

Paired mode (``--guided-dataset`` / ``--guided-checkpoint``): the Guided
codec's forward produces the hidden features the Master codec conditions on
(__main__rgbt.py:153-178); images pair by sorted file name.

  python -m compressai.utils.eval_model checkpoint DIR -a ARCH -p CKPT [-q Q] [--entropy-estimation] [--cuda]

Differences from the reference, all on the harness side: GPU timings are
synchronized; files are visited in sorted order; ``--half`` runs the
transforms in bf16 autocast (this build's reduced precision; the reference
casts to fp16); ``pretrained`` sources need network and are refused.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from collections import defaultdict
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

import compressai
from compressai.utils.metrics import ms_ssim, psnr
from compressai.zoo import load_state_dict
from compressai.zoo.image import model_architectures as architectures

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def collect_images(rootpath: str) -> List[str]:
    return sorted(os.path.join(rootpath, f) for f in os.listdir(rootpath)
                  if os.path.splitext(f)[-1].lower() in IMG_EXTENSIONS)


def read_image(filepath: str) -> torch.Tensor:
    """PIL image -> float [C, H, W] (torchvision ToTensor semantics: 8-bit images scaled to [0, 1])."""
    from PIL import Image

    if not os.path.isfile(filepath):
        raise FileNotFoundError(filepath)
    img = Image.open(filepath)
    arr = np.array(img)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    t = torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1)))
    return t.float().div(255) if arr.dtype == np.uint8 else t.float()


def _sync(x: torch.Tensor):
    if x.is_cuda:
        torch.cuda.synchronize(x.device)


def _pad(x: torch.Tensor, p: int = 64):
    """__main__t.py:106-119: centred zero padding to a multiple of p."""
    h, w = x.size(2), x.size(3)
    new_h, new_w = (h + p - 1) // p * p, (w + p - 1) // p * p
    left, top = (new_w - w) // 2, (new_h - h) // 2
    pads = (left, new_w - w - left, top, new_h - h - top)
    return F.pad(x, pads, mode="constant", value=0), pads


def _crop(x: torch.Tensor, pads):
    return F.pad(x, tuple(-p for p in pads))


def _bpp_from_likelihoods(likelihoods: Dict[str, torch.Tensor], num_pixels: int) -> float:
    return sum(torch.log(l.float()).sum() / (-math.log(2) * num_pixels) for l in likelihoods.values()).item()


def _autocast(half: bool, x: torch.Tensor):
    return torch.autocast("cuda", dtype=torch.bfloat16, enabled=bool(half and x.is_cuda))


@torch.no_grad()
def inference(model, x: torch.Tensor, half: bool = False) -> Dict[str, float]:
    """Real coding (__main__t.py:101-146)."""
    x = x.unsqueeze(0)
    x_padded, pads = _pad(x)
    _sync(x)
    start = time.time()
    with _autocast(half, x):
        out_enc = model.compress(x_padded)
    _sync(x)
    enc_time = time.time() - start
    start = time.time()
    with _autocast(half, x):
        out_dec = model.decompress(out_enc["strings"], out_enc["shape"])
    _sync(x)
    dec_time = time.time() - start
    x_hat = _crop(out_dec["x_hat"].float(), pads)
    num_pixels = x.size(0) * x.size(2) * x.size(3)
    bpp = sum(len(s[0]) for s in out_enc["strings"]) * 8.0 / num_pixels
    msssim = ms_ssim(x, x_hat, data_range=1.0).item() if min(x.shape[-2:]) > 160 else float("nan")
    return {"psnr": psnr(x, x_hat), "ms-ssim": msssim, "bpp": bpp, "encoding_time": enc_time,
            "decoding_time": dec_time}


@torch.no_grad()
def inference_entropy_estimation(model, x: torch.Tensor, half: bool = False) -> Dict[str, float]:
    """Entropy estimation (__main__t.py:149-211)."""
    x = x.unsqueeze(0)
    x_padded, pads = _pad(x)
    _sync(x)
    start = time.time()
    with _autocast(half, x):
        out_net = model.forward(x_padded)
    _sync(x)
    elapsed = time.time() - start
    num_pixels = x.size(0) * x.size(2) * x.size(3)
    bpp = _bpp_from_likelihoods(out_net["likelihoods"], num_pixels)
    x_hat = _crop(out_net["x_hat"].float(), pads)
    return {"psnr": psnr(x, x_hat), "bpp": bpp, "encoding_time": elapsed / 2.0, "decoding_time": elapsed / 2.0}


@torch.no_grad()
def inference_entropy_estimation_rgbt(model, model_guided, x: torch.Tensor, guided: torch.Tensor,
                                      half: bool = False) -> Dict[str, float]:
    """Paired entropy estimation (__main__rgbt.py:153-178): no padding (the aligners are
    built for one input size)."""
    if x.dim() == 3:
        x, guided = x.unsqueeze(0), guided.unsqueeze(0)
    _sync(x)
    start = time.time()
    with _autocast(half, x):
        hidden = model_guided(guided)["hidden"]
        out_net = model(x, guided, hidden)
    _sync(x)
    elapsed = time.time() - start
    num_pixels = x.size(0) * x.size(2) * x.size(3)
    return {"psnr": psnr(x, out_net["x_hat"].float()),
            "bpp": _bpp_from_likelihoods(out_net["likelihoods"], num_pixels),
            "encoding_time": elapsed / 2.0, "decoding_time": elapsed / 2.0}


@torch.no_grad()
def inference_rgbt(model, model_guided, x: torch.Tensor, guided: torch.Tensor) -> Dict[str, float]:
    """Paired real coding (__main__rgbt.py:99-150): the guide is coded first; the Master codec is
    conditioned on the decoded guide.  bpp counts the master's strings plus its 64 beta + 64 gamma
    fp32 side values (:142)."""
    if x.dim() == 3:
        x, guided = x.unsqueeze(0), guided.unsqueeze(0)
    _sync(x)
    start = time.time()
    out_net_r = model_guided.compress(guided)
    out_dec_r = model_guided.decompress(out_net_r["strings"], out_net_r["shape"])
    out_net = model.compress(x, out_dec_r["x_hat"])
    _sync(x)
    enc_time = time.time() - start
    start = time.time()
    out_dec = model.decompress(out_net, out_dec_r)
    _sync(x)
    dec_time = time.time() - start
    num_pixels = x.size(0) * x.size(2) * x.size(3)
    bpp = (sum(len(s[0]) for s in out_net["strings"]) * 8.0 + 64 * 2 * 4 * 8) / num_pixels
    msssim = ms_ssim(x, out_dec["x_hat"], data_range=1.0).item() if min(x.shape[-2:]) > 160 else float("nan")
    return {"psnr": psnr(x, out_dec["x_hat"]), "ms-ssim": msssim, "bpp": bpp, "encoding_time": enc_time,
            "decoding_time": dec_time}


def _state_dict_from(path: str) -> Dict[str, torch.Tensor]:
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(ckpt, dict) and "state_dict" in ckpt:
        ckpt = ckpt["state_dict"]
    return load_state_dict(ckpt)


def load_checkpoint(arch: str, checkpoint_path: str, channel: int = 3, **kwargs) -> torch.nn.Module:
    """__main__t.py:220-222, plus the fork's multi-modal classes."""
    from compressai.models import Guided_compresser, Master_compresser

    sd = _state_dict_from(checkpoint_path)
    if arch in ("Guided_compresser", "guided"):
        model = Guided_compresser(channel=channel)
        model.load_state_dict(sd)
    elif arch in ("Master_compresser", "master"):
        model = Master_compresser(width=kwargs.get("width", 256), height=kwargs.get("height", 256), channel=channel)
        model.load_state_dict(sd)
    elif arch in architectures:
        model = architectures[arch].from_state_dict(sd, channel=channel)
    else:
        raise ValueError(f'Invalid architecture "{arch}"')
    return model.eval()


def eval_model(model, filepaths, entropy_estimation=True, half=False) -> Dict[str, float]:
    """__main__t.py:226-248: metrics averaged over the images."""
    device = next(model.parameters()).device
    metrics = defaultdict(float)
    for f in filepaths:
        x = read_image(f).to(device)
        rv = inference_entropy_estimation(model, x, half) if entropy_estimation else inference(model, x, half)
        for k, v in rv.items():
            metrics[k] += v
    return {k: v / len(filepaths) for k, v in metrics.items()}


def eval_model_rgbt(model, model_guided, pairs, entropy_estimation=True, half=False) -> Dict[str, float]:
    """__main__rgbt.py:193-219."""
    device = next(model.parameters()).device
    metrics = defaultdict(float)
    for fx, fg in pairs:
        x, g = read_image(fx).to(device), read_image(fg).to(device)
        rv = (inference_entropy_estimation_rgbt(model, model_guided, x, g, half) if entropy_estimation
              else inference_rgbt(model, model_guided, x, g))
        for k, v in rv.items():
            metrics[k] += v
    return {k: v / len(pairs) for k, v in metrics.items()}


def setup_args():
    parent = argparse.ArgumentParser(add_help=False)
    parent.add_argument("dataset", type=str, help="dataset path")
    parent.add_argument("-a", "--architecture", type=str, required=True, help="model architecture")
    parent.add_argument("-c", "--entropy-coder", choices=compressai.available_entropy_coders(),
                        default=compressai.available_entropy_coders()[0], help="entropy coder (default: %(default)s)")
    parent.add_argument("--cuda", action="store_true", help="accepted for compatibility: this build always runs on the GPU")
    parent.add_argument("--half", action="store_true", help="bf16 autocast transforms")
    parent.add_argument("--entropy-estimation", action="store_true",
                        help="use evaluated entropy estimation (no entropy coding)")
    parent.add_argument("-v", "--verbose", action="store_true", help="verbose mode")
    parent.add_argument("-ch", "--channel", type=int, default=3, help="image channel")
    parent.add_argument("--guided-dataset", type=str, default=None, help="paired guide images (multi-modal codec)")
    parent.add_argument("--guided-checkpoint", type=str, default=None, help="Guided_compresser checkpoint")
    parent.add_argument("--guided-channel", type=int, default=None)
    parent.add_argument("-o", "--output", type=str, default=None, help="append the JSON result to this file")
    parser = argparse.ArgumentParser(description="Evaluate a model on an image dataset.", add_help=True)
    sub = parser.add_subparsers(help="model source", dest="source")
    pre = sub.add_parser("pretrained", parents=[parent])
    pre.add_argument("-m", "--metric", type=str, choices=["mse", "ms-ssim"], default="mse")
    pre.add_argument("-q", "--quality", dest="qualities", nargs="+", type=int, default=(1,))
    ck = sub.add_parser("checkpoint", parents=[parent])
    ck.add_argument("-p", "--path", dest="paths", type=str, nargs="*", required=True, help="checkpoint path")
    ck.add_argument("-q", "--quality", dest="quality", type=int, help="quality")
    return parser


def main(argv):
    parser = setup_args()
    args = parser.parse_args(argv)
    if not args.source:
        print("Error: missing 'checkpoint' or 'pretrained' source.", file=sys.stderr)
        parser.print_help()
        raise SystemExit(1)
    if args.source == "pretrained":
        print("Error: pretrained weights are remote downloads; use a checkpoint.", file=sys.stderr)
        raise SystemExit(1)
    filepaths = collect_images(args.dataset)
    if len(filepaths) == 0:
        print("Error: no images found in directory.", file=sys.stderr)
        raise SystemExit(1)
    compressai.set_entropy_coder(args.entropy_coder)
    if not torch.cuda.is_available():
        raise SystemExit("eval_model: this build runs on the GPU only (MI355X HIP kernels) and no GPU is visible")
    device = "cuda"
    paired = args.guided_dataset is not None
    results = defaultdict(list)
    for run in args.paths:
        if args.verbose:
            sys.stderr.write(f"\rEvaluating {run}")
            sys.stderr.flush()
        if paired:
            gfiles = collect_images(args.guided_dataset)
            if len(gfiles) != len(filepaths):
                raise SystemExit("Error: guided and master directories hold different image counts.")
            h, w = read_image(filepaths[0]).shape[-2:]
            model = load_checkpoint(args.architecture, run, args.channel, width=w, height=h).to(device)
            gch = args.guided_channel or (3 if args.channel == 1 else 1)
            model_g = load_checkpoint("Guided_compresser", args.guided_checkpoint, gch).to(device)
            if not args.entropy_estimation:
                model.update()
                model_g.update()
            metrics = eval_model_rgbt(model, model_g, list(zip(filepaths, gfiles)), args.entropy_estimation,
                                      args.half)
        else:
            model = load_checkpoint(args.architecture, run, args.channel).to(device)
            if not args.entropy_estimation:
                model.update()
            metrics = eval_model(model, filepaths, args.entropy_estimation, args.half)
        for k, v in metrics.items():
            results[k].append(v)
    if args.verbose:
        sys.stderr.write("\n")
    description = "entropy estimation" if args.entropy_estimation else args.entropy_coder
    output = {"name": args.architecture, "description": f"Inference ({description})", "results": results}
    if args.output:
        with open(args.output, "a") as f:
            f.write(json.dumps(output) + "\n")
    print(json.dumps(output, indent=2))
    return output


if __name__ == "__main__":
    main(sys.argv[1:])
