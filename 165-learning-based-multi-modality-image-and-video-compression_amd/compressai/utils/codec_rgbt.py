"""The multi-modal bit-stream container and its image encode / decode CLI (reference: examples/codec_rgbt.py:
141-386, 454-555, 607-830).

File layout, all integers big-endian (codec_rgbt.py:188-250, 328-386):

    u8  model id             index of the architecture in the reference's model registry (``MODEL_IDS``)
    u8  code                 metric << 4 | (quality - 1) & 0x0F
    u32 height, u32 width    original image size
    u8  bitdepth             8
    [f32 x 64 beta, f32 x 64 gamma]      Master_compresser only: the channel aligner's side information
    u32 shape[0], u32 shape[1], u32 n    latent grid of the hyper-latent z and the number of strings
    n x (u32 length, bytes)              the y string, then the z string (first image of the batch)

The multi-modal decoder needs the guide modality's reconstruction: as in the reference, the guide image is coded
and decoded again with the ``Guided_compresser`` on both sides (codec_rgbt.py:350-356, 538-545), so the file
holds the master's bits only.

    python -m compressai.utils.codec_rgbt encode IMG --model Master_compresser --path G.pth M.pth -ch 3 -o out.bin
    python -m compressai.utils.codec_rgbt decode out.bin --model Master_compresser --path G.pth M.pth \
        -ch 3 --guided GUIDE_IMG -o rec.png
"""
from __future__ import annotations

import argparse
import struct
import sys
import time
from pathlib import Path
from typing import IO, Dict, List, NamedTuple, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

# the reference's registry order: compressai.zoo.models (6 image models + ssf2020), then the two multi-modal
# codecs appended by codec_rgbt.py:66-69.  Ids are part of the file format, so they are spelled out.
MODEL_IDS: Dict[str, int] = {
    "bmshj2018-factorized": 0, "bmshj2018-hyperprior": 1, "mbt2018-mean": 2, "mbt2018": 3,
    "cheng2020-anchor": 4, "cheng2020-attn": 5, "ssf2020": 6, "Master_compresser": 7, "Guided_compresser": 8,
}
METRIC_IDS: Dict[str, int] = {"mse": 0, "ms-ssim": 1}
SIDE_CHANNELS = 64    # beta / gamma floats per image (codec_rgbt.py:513-514)
BITDEPTH = 8


# ---------------------------------------------------------------------------------------------------------
# primitive big-endian fields (codec_rgbt.py:141-185)

def write_uints(fd: IO[bytes], values: Sequence[int]) -> int:
    fd.write(struct.pack(f">{len(values)}I", *values))
    return 4 * len(values)


def read_uints(fd: IO[bytes], n: int) -> Tuple[int, ...]:
    return struct.unpack(f">{n}I", _read_exact(fd, 4 * n))


def write_uchars(fd: IO[bytes], values: Sequence[int]) -> int:
    fd.write(struct.pack(f">{len(values)}B", *values))
    return len(values)


def read_uchars(fd: IO[bytes], n: int) -> Tuple[int, ...]:
    return struct.unpack(f">{n}B", _read_exact(fd, n))


def write_floats(fd: IO[bytes], values: Sequence[float]) -> int:
    fd.write(struct.pack(f">{len(values)}f", *values))
    return 4 * len(values)


def read_floats(fd: IO[bytes], n: int) -> Tuple[float, ...]:
    return struct.unpack(f">{n}f", _read_exact(fd, 4 * n))


def write_bytes(fd: IO[bytes], values: bytes) -> int:
    fd.write(values)
    return len(values)


def read_bytes(fd: IO[bytes], n: int) -> bytes:
    return _read_exact(fd, n)


def _read_exact(fd: IO[bytes], n: int) -> bytes:
    b = fd.read(n)
    if len(b) != n:
        raise ValueError(f"truncated bit-stream: wanted {n} bytes, got {len(b)}")
    return b


# ---------------------------------------------------------------------------------------------------------
# header and body (codec_rgbt.py:188-250)

def get_header(model_name: str, metric: str, quality: int) -> Tuple[int, int]:
    """(model id, metric << 4 | quality - 1) -- two bytes (codec_rgbt.py:188-203)."""
    if model_name not in MODEL_IDS:
        raise ValueError(f'unknown model "{model_name}"')
    if metric not in METRIC_IDS:
        raise ValueError(f'unknown metric "{metric}"')
    if not 1 <= quality <= 16:
        raise ValueError(f"quality {quality} does not fit the 4-bit field")
    return MODEL_IDS[model_name], (METRIC_IDS[metric] << 4) | ((quality - 1) & 0x0F)


def parse_header(header: Sequence[int]) -> Tuple[str, str, int]:
    """(model name, metric, quality) from the two header bytes (codec_rgbt.py:206-221)."""
    model_id, code = header
    names = {v: k for k, v in MODEL_IDS.items()}
    metrics = {v: k for k, v in METRIC_IDS.items()}
    if model_id not in names or (code >> 4) not in metrics:
        raise ValueError(f"bad header {tuple(header)}")
    return names[model_id], metrics[code >> 4], (code & 0x0F) + 1


def write_body(fd: IO[bytes], shape: Sequence[int], out_strings: Sequence[Sequence[bytes]]) -> int:
    """Latent shape, string count, then each string's first-image bytes length-prefixed (codec_rgbt.py:239-249)."""
    n = write_uints(fd, (int(shape[0]), int(shape[1]), len(out_strings)))
    for s in out_strings:
        n += write_uints(fd, (len(s[0]),))
        n += write_bytes(fd, s[0])
    return n


def read_body(fd: IO[bytes]) -> Tuple[List[List[bytes]], Tuple[int, int]]:
    """Inverse of write_body: ([[y bytes], [z bytes]], shape) (codec_rgbt.py:224-235)."""
    shape = read_uints(fd, 2)
    n_strings = read_uints(fd, 1)[0]
    strings = [[read_bytes(fd, read_uints(fd, 1)[0])] for _ in range(n_strings)]
    return strings, shape


class Header(NamedTuple):
    model: str
    metric: str
    quality: int
    original_size: Tuple[int, int]
    bitdepth: int


def write_stream(fd: IO[bytes], model: str, metric: str, quality: int, original_size: Sequence[int], out: Dict,
                 bitdepth: int = BITDEPTH) -> int:
    """One coded image: header, size, bitdepth, [beta, gamma], body (codec_rgbt.py:369-382)."""
    n = write_uchars(fd, get_header(model, metric, quality))
    n += write_uints(fd, (int(original_size[0]), int(original_size[1])))
    n += write_uchars(fd, (bitdepth,))
    if model == "Master_compresser":
        for key in ("beta", "gamma"):
            v = out[key][:1].reshape(-1).float().cpu().tolist()
            if len(v) != SIDE_CHANNELS:
                raise ValueError(f"{key} has {len(v)} values, the container holds {SIDE_CHANNELS}")
            n += write_floats(fd, v)
    n += write_body(fd, out["shape"], out["strings"])
    return n


def read_stream(fd: IO[bytes]) -> Tuple[Header, Dict]:
    """Inverse of write_stream: the header and the ``out_net`` dict decompress() takes (codec_rgbt.py:511-523,
    616-620)."""
    model, metric, quality = parse_header(read_uchars(fd, 2))
    size = read_uints(fd, 2)
    bitdepth = read_uchars(fd, 1)[0]
    out: Dict = {}
    if model == "Master_compresser":
        out["beta"] = torch.tensor(read_floats(fd, SIDE_CHANNELS)).reshape(1, SIDE_CHANNELS, 1, 1)
        out["gamma"] = torch.tensor(read_floats(fd, SIDE_CHANNELS)).reshape(1, SIDE_CHANNELS, 1, 1)
    out["strings"], out["shape"] = read_body(fd)
    return Header(model, metric, quality, (size[0], size[1]), bitdepth), out


# ---------------------------------------------------------------------------------------------------------
# image I/O (codec_rgbt.py:134-138, 279-307)

def img2torch(img, device) -> torch.Tensor:
    from compressai.datasets._functional import to_tensor

    return to_tensor(img).unsqueeze(0).to(device)


def torch2img(x: torch.Tensor):
    """ToPILImage on a [0, 1] float tensor: x * 255 truncated to uint8; 1 channel -> mode "L"."""
    from PIL import Image

    a = (x.detach().clamp(0, 1).squeeze(0) * 255).to(torch.uint8).cpu().numpy()
    return Image.fromarray(a[0], mode="L") if a.shape[0] == 1 else Image.fromarray(a.transpose(1, 2, 0))


def pad(x: torch.Tensor, p: int = 64) -> torch.Tensor:
    h, w = x.size(2), x.size(3)
    H, W = (h + p - 1) // p * p, (w + p - 1) // p * p
    left, top = (W - w) // 2, (H - h) // 2
    return F.pad(x, (left, W - w - left, top, H - h - top), mode="constant", value=0)


def crop(x: torch.Tensor, size: Sequence[int]) -> torch.Tensor:
    H, W = x.size(2), x.size(3)
    h, w = size
    left, top = (W - w) // 2, (H - h) // 2
    return F.pad(x, (-left, -(W - w - left), -top, -(H - h - top)), mode="constant", value=0)


def guide_path_for(master_path: str, channel: int) -> str:
    """The co-located frame of the other modality (codec_rgbt.py:331-341)."""
    if channel == 3:
        return master_path.replace("RGB", "thermal_8_bit").replace("jpg", "jpeg")
    return master_path.replace("thermal_8_bit", "RGB").replace("jpeg", "jpg")


def load_master_image(path: str, channel: int, device) -> torch.Tensor:
    from PIL import Image

    from compressai.datasets.image import FLIR_RGB_SIZE

    img = Image.open(path)
    if channel == 3:
        img = img.convert("RGB").resize(FLIR_RGB_SIZE)
    return img2torch(img, device)


def load_guide_image(path: str, channel: int, device) -> torch.Tensor:
    """``channel`` is the master's: an RGB master is guided by the thermal frame as stored, a thermal master
    by the RGB frame resized to 1280x1024 (codec_rgbt.py:333-341)."""
    from PIL import Image

    from compressai.datasets.image import FLIR_RGB_SIZE

    img = Image.open(path)
    if channel != 3:
        img = img.convert("RGB").resize(FLIR_RGB_SIZE)
    return img2torch(img, device)


# ---------------------------------------------------------------------------------------------------------
# codec (codec_rgbt.py:328-386, 511-555)

def _guide_reconstruction(model_guided, guided: torch.Tensor) -> Dict:
    enc = model_guided.compress(guided)
    return model_guided.decompress(enc["strings"], enc["shape"])


@torch.no_grad()
def encode_image(x: torch.Tensor, net, output: str, model: str, metric: str = "mse", quality: int = 3,
                 guided: Optional[torch.Tensor] = None) -> Dict[str, float]:
    """Code ``x`` [1, C, H, W] into ``output``.  ``net`` is a model, or ``[Guided_compresser, Master_compresser]``
    with ``guided`` the guide-modality image.  Returns the file's bpp (codec_rgbt.py:384-386)."""
    h, w = x.size(2), x.size(3)
    if isinstance(net, (list, tuple)):
        if guided is None:
            raise ValueError("Master_compresser needs the guide image")
        model_guided, master = net
        out = master.compress(x, _guide_reconstruction(model_guided, guided)["x_hat"])
    else:
        out = net.compress(x)
    with Path(output).open("wb") as f:
        write_stream(f, model, metric, quality, (h, w), out)
    return {"bpp": Path(output).stat().st_size * 8.0 / (h * w)}


@torch.no_grad()
def decode_image(inputpath: str, net, guided: Optional[torch.Tensor] = None) -> Tuple[Header, torch.Tensor]:
    """Decode ``inputpath`` to the [1, C, H, W] reconstruction in [0, 1] (codec_rgbt.py:511-555)."""
    with Path(inputpath).open("rb") as f:
        hdr, out = read_stream(f)
    if isinstance(net, (list, tuple)):
        if hdr.model != "Master_compresser":
            raise ValueError(f"stream was coded with {hdr.model}, not Master_compresser")
        if guided is None:
            raise ValueError("Master_compresser needs the guide image")
        model_guided, master = net
        dev = next(master.parameters()).device
        out["beta"], out["gamma"] = out["beta"].to(dev), out["gamma"].to(dev)
        x_hat = master.decompress(out, _guide_reconstruction(model_guided, guided))["x_hat"]
    else:
        x_hat = net.decompress(out["strings"], out["shape"])["x_hat"]
    return hdr, crop(x_hat, hdr.original_size)


def _device(args) -> str:
    """This build's kernels are GPU-only: the CLIs always use the GPU and fail up front without one."""
    if not torch.cuda.is_available():
        raise SystemExit("codec_rgbt: this build runs on the GPU only (MI355X HIP kernels) and no GPU is visible")
    return "cuda"


def _load_nets(model: str, paths: Sequence[str], channel: int, device):
    from compressai.utils.eval_model.__main__ import load_checkpoint

    if model == "Master_compresser":
        if len(paths) != 2:
            raise ValueError("Master_compresser takes two checkpoints: the guide's, then the master's")
        guided_chl = 1 if channel == 3 else 3
        g = load_checkpoint("Guided_compresser", paths[0], channel=guided_chl).to(device)
        m = load_checkpoint("Master_compresser", paths[1], channel=channel, width=512, height=640).to(device)
        nets = [g, m]
    else:
        nets = [load_checkpoint(model, paths[0], channel=channel).to(device)]
    for n in nets:
        n.update()
    return nets if model == "Master_compresser" else nets[0]


def _common_args(p: argparse.ArgumentParser):
    p.add_argument("--model", default="Guided_compresser", choices=list(MODEL_IDS))
    p.add_argument("--path", required=True, nargs="+", help="checkpoint path(s): guide then master")
    p.add_argument("-ch", "--channel", type=int, default=3, help="master image channels")
    p.add_argument("--guided", default=None, help="guide-modality image (default: derived from the input path)")
    p.add_argument("-c", "--coder", default="ans")
    p.add_argument("--cuda", action="store_true", help="accepted for compatibility: this build always runs on the GPU")
    p.add_argument("-o", "--output", required=True)


def encode(argv):
    import compressai

    p = argparse.ArgumentParser(description="Encode an image to a bit-stream")
    p.add_argument("input")
    p.add_argument("-m", "--metric", choices=list(METRIC_IDS), default="mse")
    p.add_argument("-q", "--quality", type=int, default=3)
    _common_args(p)
    a = p.parse_args(argv)
    compressai.set_entropy_coder(a.coder)
    device = _device(a)
    net = _load_nets(a.model, a.path, a.channel, device)
    x = load_master_image(a.input, a.channel, device)
    guided = None
    if a.model == "Master_compresser":
        guided = load_guide_image(a.guided or guide_path_for(a.input, a.channel), a.channel, device)
    t = time.time()
    r = encode_image(x, net, a.output, a.model, a.metric, a.quality, guided)
    print(f"{r['bpp']:.3f} bpp | Encoded in {time.time() - t:.2f}s")


def decode(argv):
    import compressai

    p = argparse.ArgumentParser(description="Decode a bit-stream to an image")
    p.add_argument("input")
    _common_args(p)
    a = p.parse_args(argv)
    compressai.set_entropy_coder(a.coder)
    device = _device(a)
    net = _load_nets(a.model, a.path, a.channel, device)
    guided = None
    if a.model == "Master_compresser":
        if a.guided is None:
            raise SystemExit("--guided is required to decode a Master_compresser stream")
        guided = load_guide_image(a.guided, a.channel, device)
    t = time.time()
    _, x_hat = decode_image(a.input, net, guided)
    torch2img(x_hat).save(a.output)
    print(f"Decoded in {time.time() - t:.2f}s")


def main(argv):
    if not argv or argv[0] not in ("encode", "decode"):
        raise SystemExit("usage: python -m compressai.utils.codec_rgbt {encode,decode} ...")
    (encode if argv[0] == "encode" else decode)(argv[1:])


if __name__ == "__main__":
    main(sys.argv[1:])
