from .conv import Conv2d, ConvTranspose2d, Sequential
from .gdn import GDN, GDN1
from .layers import MaskedConv2d, conv1x1, conv3x3

__all__ = ["Conv2d", "ConvTranspose2d", "Sequential", "GDN", "GDN1", "MaskedConv2d", "conv1x1", "conv3x3"]
