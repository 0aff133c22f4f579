from .conv import Conv2d, ConvTranspose2d, PixelShuffle, Sequential
from .gdn import GDN, GDN1
from .layers import (AttentionBlock, MaskedConv2d, ResidualBlock, ResidualBlockUpsample, ResidualBlockWithStride,
                     ResidualUnit, conv1x1, conv3x3, subpel_conv3x3)

__all__ = ["Conv2d", "ConvTranspose2d", "PixelShuffle", "Sequential", "GDN", "GDN1", "MaskedConv2d", "conv1x1",
           "conv3x3", "subpel_conv3x3", "ResidualBlockWithStride", "ResidualBlockUpsample", "ResidualBlock",
           "ResidualUnit", "AttentionBlock"]
