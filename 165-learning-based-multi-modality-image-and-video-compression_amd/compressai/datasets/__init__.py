"""Image datasets (reference: compressai/datasets/__init__.py:30-40).

Only the still-image loaders the training / eval path reads are provided: the plain ``ImageFolder``
and the paired FLIR RGB + thermal loaders.  The video loaders (``VideoFolder``, ``RawVideoSequence``)
belong to the reference's video codecs, which are outside this package's scope.
"""
from .image import TEST_TRANSFORM, TRAIN_TRANSFORM, ImageFolder
from .image_rgbt import (FLIR_TEST_LIST, ImageFolderRGB, ImageFolderT, ImageFolderTest, guided_dir,
                         paired_random_crop, paired_train_transforms)

__all__ = ["ImageFolder", "ImageFolderRGB", "ImageFolderT", "ImageFolderTest", "TEST_TRANSFORM",
           "TRAIN_TRANSFORM", "FLIR_TEST_LIST", "guided_dir", "paired_random_crop", "paired_train_transforms"]
