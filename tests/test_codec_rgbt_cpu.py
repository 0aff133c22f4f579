"""Multi-modal container format (examples/codec_rgbt.py:141-386) and the paired FLIR loaders
(datasets/image_rgbt_rgb.py:40-150, image_rgbt_t.py, image_rgbt_test.py) -- host code, no GPU."""
import io
import struct

import numpy as np
import pytest
import torch


def _out(master: bool):
    g = torch.Generator().manual_seed(3)
    out = {"strings": [[bytes(range(7)) * 3], [b"\x00\xffz"]], "shape": torch.Size([4, 5])}
    if master:
        out["beta"] = torch.randn(1, 64, 1, 1, generator=g)
        out["gamma"] = torch.randn(1, 64, 1, 1, generator=g)
    return out


def test_header_fields():
    from compressai.utils.codec_rgbt import get_header, parse_header

    # ids follow the reference's registry: zoo.models (7 entries incl. ssf2020) then Master, Guided
    assert get_header("Master_compresser", "mse", 3) == (7, 2)
    assert get_header("Guided_compresser", "ms-ssim", 8) == (8, 0x17)
    assert get_header("bmshj2018-hyperprior", "mse", 1) == (1, 0)
    for name, metric, q in [("Master_compresser", "mse", 3), ("cheng2020-attn", "ms-ssim", 16)]:
        assert parse_header(get_header(name, metric, q)) == (name, metric, q)
    with pytest.raises(ValueError):
        get_header("Master_compresser", "mse", 17)
    with pytest.raises(ValueError):
        parse_header((42, 0))


@pytest.mark.parametrize("master", [False, True])
def test_stream_byte_layout(master):
    """The exact bytes of codec_rgbt.py:369-382: big-endian u8/u32/f32 fields in order."""
    from compressai.utils.codec_rgbt import read_stream, write_stream

    out = _out(master)
    model = "Master_compresser" if master else "Guided_compresser"
    buf = io.BytesIO()
    n = write_stream(buf, model, "mse", 3, (1024, 1280), out)
    b = buf.getvalue()
    assert n == len(b)
    exp = struct.pack(">2B", 7 if master else 8, 2) + struct.pack(">2I", 1024, 1280) + struct.pack(">B", 8)
    if master:
        exp += struct.pack(">64f", *out["beta"].flatten().tolist()) + struct.pack(">64f", *out["gamma"].flatten().tolist())
    exp += struct.pack(">3I", 4, 5, 2)
    for s in out["strings"]:
        exp += struct.pack(">I", len(s[0])) + s[0]
    assert b == exp

    hdr, back = read_stream(io.BytesIO(b))
    assert hdr == (model, "mse", 3, (1024, 1280), 8)
    assert back["strings"] == out["strings"] and tuple(back["shape"]) == (4, 5)
    if master:
        # fp32 side information travels losslessly
        assert torch.equal(back["beta"], out["beta"]) and torch.equal(back["gamma"], out["gamma"])


def test_truncated_stream_raises():
    from compressai.utils.codec_rgbt import read_stream, write_stream

    buf = io.BytesIO()
    write_stream(buf, "Master_compresser", "mse", 3, (64, 64), _out(True))
    b = buf.getvalue()
    for cut in (1, 5, 100, len(b) - 1):
        with pytest.raises(ValueError):
            read_stream(io.BytesIO(b[:cut]))


def test_side_information_size_checked():
    from compressai.utils.codec_rgbt import write_stream

    out = _out(True)
    out["beta"] = torch.zeros(1, 32, 1, 1)
    with pytest.raises(ValueError):
        write_stream(io.BytesIO(), "Master_compresser", "mse", 3, (64, 64), out)


def test_pad_crop_and_image_conversion():
    from compressai.utils.codec_rgbt import crop, img2torch, pad, torch2img

    x = torch.rand(1, 3, 70, 131, generator=torch.Generator().manual_seed(0))
    xp = pad(x)
    assert xp.shape[-2:] == (128, 192)
    assert torch.equal(crop(xp, (70, 131)), x)
    q = (x * 255).floor() / 255
    assert torch.allclose(img2torch(torch2img(q), "cpu"), q, atol=1e-6)
    g = torch.rand(1, 1, 8, 9)
    assert torch2img(g).mode == "L"


def test_guide_path_derivation():
    from compressai.utils.codec_rgbt import guide_path_for

    assert guide_path_for("/d/val/RGB/FLIR_08884.jpg", 3) == "/d/val/thermal_8_bit/FLIR_08884.jpeg"
    assert guide_path_for("/d/val/thermal_8_bit/FLIR_08884.jpeg", 1) == "/d/val/RGB/FLIR_08884.jpg"


# ------------------------------------------------------------------------------------------------- datasets

def _ramp(h, w):
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    return (0.7 * xx + 0.3 * yy) * 255


def _flir(tmp_path, n=3, th=(96, 120)):
    """A synthetic FLIR split: RGB at 2x the thermal resolution, both the same ramp (different per frame)."""
    from PIL import Image

    rgb, thermal = tmp_path / "val" / "RGB", tmp_path / "val" / "thermal_8_bit"
    rgb.mkdir(parents=True)
    thermal.mkdir(parents=True)
    for i in range(n):
        t = _ramp(*th)
        if i % 2:
            t = t[:, ::-1]
        Image.fromarray(t.astype(np.uint8), mode="L").save(thermal / f"FLIR_{i:05d}.png")
        r = np.kron(t, np.ones((2, 2)))
        Image.fromarray(np.repeat(r[:, :, None], 3, 2).astype(np.uint8)).save(rgb / f"FLIR_{i:05d}.png")
    return rgb, thermal


def test_paired_rgb_master_colocated(tmp_path):
    """RGB master: the crop windows are co-located and flipped together (image_rgbt_rgb.py:40-77)."""
    import random

    import torch.nn.functional as F

    from compressai.datasets import ImageFolderRGB

    rgb, _ = _flir(tmp_path)
    ds = ImageFolderRGB(str(rgb), channel=3, crop_size=(48, 64))
    assert len(ds) == 3
    random.seed(0)
    flips = 0
    for k in range(12):
        img, guided = ds[k % 3]
        assert img.shape == (3, 96, 128) and guided.shape == (1, 48, 64)
        down = F.avg_pool2d(img[None, :1], 2)[0]
        assert (down - guided).abs().mean() < 0.02
        assert (down - guided.flip(-1)).abs().mean() > 0.05      # a lone flip would be caught
        flips += int(guided[0, :, 0].mean() > guided[0, :, -1].mean()) ^ (k % 3 == 1)
    assert 0 < flips < 12


def test_paired_thermal_master(tmp_path):
    import random

    from compressai.datasets import ImageFolderRGB

    _, thermal = _flir(tmp_path)
    ds = ImageFolderRGB(str(thermal), channel=1)
    random.seed(1)
    img, guided = ds[0]
    assert img.shape == (1, 96, 120) and guided.shape == (3, 1024, 1280)


def test_single_modality_and_test_loaders(tmp_path):
    from PIL import Image

    from compressai.datasets import TEST_TRANSFORM, ImageFolder, ImageFolderT, ImageFolderTest

    rgb, thermal = _flir(tmp_path, n=2)
    t = ImageFolderT(str(thermal), channel=1)
    assert len(t) == 2 and t[0].shape == (1, 96, 120)
    r = ImageFolderT(str(rgb), channel=3)
    assert r[1].shape == (3, 1024, 1280)
    f = ImageFolder(str(tmp_path / "val"), transform=TEST_TRANSFORM, split="RGB", size=(256, 320))
    assert f[0].shape == (3, 256, 320)
    # the fixed evaluation list, with the reference's file extensions
    for i, name in enumerate(("FLIR_08884", "FLIR_09042")):
        Image.open(rgb / f"FLIR_{i:05d}.png").save(rgb / f"{name}.jpg")
        Image.open(thermal / f"FLIR_{i:05d}.png").save(thermal / f"{name}.jpeg")
    te = ImageFolderTest(str(rgb), channel=3, names=("FLIR_08884", "FLIR_09042"))
    x, g = te[1]
    assert x.shape == (3, 1024, 1280) and g.shape == (1, 96, 120)
    assert te.pairs()[0][1].endswith("thermal_8_bit/FLIR_08884.jpeg")
    with pytest.raises(RuntimeError):
        ImageFolderRGB_missing = ImageFolderTest(str(tmp_path / "nope" / "RGB"))    # noqa: F841
