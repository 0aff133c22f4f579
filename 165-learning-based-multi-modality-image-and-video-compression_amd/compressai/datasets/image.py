"""Single-modality image folder (reference: compressai/datasets/image.py:45-120)."""
from __future__ import annotations

import random
from pathlib import Path

from PIL import Image, ImageFile
from torch.utils.data import Dataset

from ._functional import center_crop, hflip, to_tensor

ImageFile.LOAD_TRUNCATED_IMAGES = True    # image.py:43: some FLIR frames are truncated JPEGs

TEST_TRANSFORM = 1    # image.py:38-39
TRAIN_TRANSFORM = 2

FLIR_RGB_SIZE = (1280, 1024)    # PIL (width, height) every RGB frame is resized to (image.py:113)


class ImageFolder(Dataset):
    """``root/split/*`` images, each converted to ``mode`` and resized to 1280x1024 (image.py:90-120).

    ``transform`` is ``TRAIN_TRANSFORM`` (random horizontal flip, image.py:50-63), ``TEST_TRANSFORM``
    (centre crop to ``size``, image.py:65-66), any callable, or None (the PIL image itself).
    """

    def __init__(self, root, transform=None, split="train", size=(224, 224), mode="RGB"):
        splitdir = Path(root) / split if split else Path(root)
        if not splitdir.is_dir():
            raise RuntimeError(f'Invalid directory "{root}"')
        self.samples = sorted(f for f in splitdir.iterdir() if f.is_file())
        self.transform = transform
        self.size = size
        self.mode = mode

    def __getitem__(self, index):
        img = Image.open(self.samples[index]).convert(self.mode).resize(FLIR_RGB_SIZE)
        if self.transform == TEST_TRANSFORM:
            return center_crop(to_tensor(img), self.size)
        if self.transform == TRAIN_TRANSFORM:
            x = to_tensor(img)
            return hflip(x) if random.random() < 0.5 else x
        if callable(self.transform):
            return self.transform(img)
        return img

    def __len__(self):
        return len(self.samples)
