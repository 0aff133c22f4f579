"""Paired FLIR RGB + thermal loaders (reference: compressai/datasets/image_rgbt_rgb.py:40-150,
image_rgbt_t.py:57-100, image_rgbt_test.py:40-125).

FLIR ADAS keeps the two modalities in sibling directories whose names differ only in the modality:
``.../RGB/FLIR_xxxxx.jpg`` (1800x1600 colour) and ``.../thermal_8_bit/FLIR_xxxxx.jpeg`` (640x512, mode "L").
The master image is the one being coded; the guide is the other modality, coded first.

* master RGB (``channel=3``): the thermal guide sets the geometry.  ``paired_train_transforms`` scales the
  guide by a random factor from ``TRAIN_SCALES``, the RGB image to exactly twice the guide's size, crops a
  512x640 guide window and the co-located 1024x1280 RGB window, and flips both together;
* master thermal (``channel=1``): the RGB guide is resized to 1280x1024; both are flipped together.

Every sample is a ``(master, guide)`` pair of float CHW tensors in [0, 1].
"""
from __future__ import annotations

import random
from pathlib import Path
from typing import Tuple

import torch
from PIL import Image, ImageFile
from torch.utils.data import Dataset

from ._functional import hflip, resize, to_tensor
from .image import FLIR_RGB_SIZE

ImageFile.LOAD_TRUNCATED_IMAGES = True

TRAIN_SCALES = (1, 1.2, 1.4, 1.6, 1.8)    # image_rgbt_rgb.py:49

# the 20 FLIR validation frames the reference reports on (image_rgbt_test.py:40-61)
FLIR_TEST_LIST = (
    "FLIR_08884", "FLIR_09042", "FLIR_09063", "FLIR_09175", "FLIR_09218", "FLIR_09311", "FLIR_09451",
    "FLIR_09673", "FLIR_09682", "FLIR_09705", "FLIR_09706", "FLIR_09728", "FLIR_09751", "FLIR_09792",
    "FLIR_09886", "FLIR_09896", "FLIR_10082", "FLIR_10107", "FLIR_10171", "FLIR_10217",
)


def guided_dir(root: str, channel: int) -> Path:
    """The guide modality's directory (image_rgbt_rgb.py:104-107)."""
    return Path(root.replace("RGB", "thermal_8_bit") if channel == 3 else root.replace("thermal_8_bit", "RGB"))


def paired_random_crop(img: torch.Tensor, guided: torch.Tensor, height: int, width: int
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """A height x width guide window and the co-located 2x window of the master (image_rgbt_rgb.py:40-46)."""
    if guided.shape[1] < height or guided.shape[2] < width:
        raise ValueError(f"guide {tuple(guided.shape[1:])} is smaller than the crop {(height, width)}")
    y = random.randint(0, guided.shape[1] - height)
    x = random.randint(0, guided.shape[2] - width)
    return img[:, 2 * y:2 * (y + height), 2 * x:2 * (x + width)], guided[:, y:y + height, x:x + width]


def paired_train_transforms(img, guided, crop_size=(512, 640)) -> Tuple[torch.Tensor, torch.Tensor]:
    """Random rescale, co-located crop and joint flip (image_rgbt_rgb.py:51-77).  ``img`` and ``guided``
    are PIL images or CHW tensors in [0, 1]; the master comes out at twice the guide's resolution."""
    guided = guided if torch.is_tensor(guided) else to_tensor(guided)
    img = img if torch.is_tensor(img) else to_tensor(img)
    scale = random.choice(TRAIN_SCALES)
    sh, sw = int(guided.shape[1] * scale), int(guided.shape[2] * scale)
    guided = resize(guided, (sh, sw))
    img = resize(img, (2 * sh, 2 * sw))
    img, guided = paired_random_crop(img, guided, crop_size[0], crop_size[1])
    if random.random() > 0.5:
        guided, img = hflip(guided), hflip(img)
    return img, guided


def _files(d: Path):
    return sorted(f for f in d.iterdir() if f.is_file())


class ImageFolderRGB(Dataset):
    """Paired training loader (image_rgbt_rgb.py:80-150).  ``root`` is the master modality's directory;
    the guide's directory is derived by ``guided_dir``; files pair up by sorted order."""

    def __init__(self, root, size=(224, 224), channel=3, crop_size=(512, 640)):
        self.root = root
        splitdir, gdir = Path(root), guided_dir(str(root), channel)
        if not splitdir.is_dir() or not gdir.is_dir():
            raise RuntimeError(f'Invalid directory "{root}"')
        self.samples = _files(splitdir)
        self.guided_samples = _files(gdir)
        self.size = size
        self.channel = channel
        self.crop_size = crop_size

    def __getitem__(self, index):
        if self.channel == 3:
            img = Image.open(self.samples[index]).convert("RGB")
            guided = Image.open(self.guided_samples[index])
            return paired_train_transforms(img, guided, self.crop_size)
        img = to_tensor(Image.open(self.samples[index]))
        guided = to_tensor(Image.open(self.guided_samples[index]).convert("RGB").resize(FLIR_RGB_SIZE))
        if random.random() > 0.5:
            guided, img = hflip(guided), hflip(img)
        return img, guided

    def __len__(self):
        # the two modality folders are not the same size in FLIR (image_rgbt_rgb.py:145-149)
        return len(self.samples) if self.channel == 3 else len(self.guided_samples)


class ImageFolderT(Dataset):
    """Single-modality loader used to train the guide codec (image_rgbt_t.py:57-100): RGB frames resized to
    1280x1024 (``channel=3``) or thermal frames as mode "L" (``channel=1``), randomly flipped."""

    def __init__(self, root, size=(224, 224), channel=3):
        splitdir = Path(root)
        if not splitdir.is_dir():
            raise RuntimeError(f'Invalid directory "{root}"')
        self.samples = _files(splitdir)
        self.size = size
        self.channel = channel

    def __getitem__(self, index):
        if self.channel == 3:
            x = to_tensor(Image.open(self.samples[index]).convert("RGB").resize(FLIR_RGB_SIZE))
        else:
            x = to_tensor(Image.open(self.samples[index]).convert("L"))
        return hflip(x) if random.random() < 0.5 else x

    def __len__(self):
        return len(self.samples)


class ImageFolderTest(Dataset):
    """The fixed 20-frame FLIR evaluation pairs (image_rgbt_test.py:64-125): no augmentation; the RGB side
    is resized to 1280x1024, the thermal side kept at 640x512."""

    def __init__(self, root, size=(224, 224), channel=3, names=FLIR_TEST_LIST):
        splitdir, gdir = Path(root), guided_dir(str(root), channel)
        if not splitdir.is_dir() or not gdir.is_dir():
            raise RuntimeError(f'Invalid directory "{root}"')
        ext, gext = (".jpg", ".jpeg") if channel == 3 else (".jpeg", ".jpg")
        self.samples = [splitdir / (n + ext) for n in names]
        self.guided_samples = [gdir / (n + gext) for n in names]
        self.size = size
        self.channel = channel

    def pairs(self):
        """(master path, guide path) per frame -- the input of eval_model_rgbt."""
        return [(str(a), str(b)) for a, b in zip(self.samples, self.guided_samples)]

    def __getitem__(self, index):
        if self.channel == 3:
            img = Image.open(self.samples[index]).convert("RGB").resize(FLIR_RGB_SIZE)
            guided = Image.open(self.guided_samples[index])
        else:
            img = Image.open(self.samples[index])
            guided = Image.open(self.guided_samples[index]).convert("RGB").resize(FLIR_RGB_SIZE)
        return to_tensor(img), to_tensor(guided)

    def __len__(self):
        return len(self.samples)
