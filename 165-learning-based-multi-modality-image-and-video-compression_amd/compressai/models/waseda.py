"""cheng2020 models (reference: compressai/models/waseda.py:48-158).

Cheng2020Anchor / Cheng2020Attention on the HIP path: residual blocks with
3x3 / 1x1 convs, GDN / IGDN, sub-pixel upsampling and (Attention) gated
residual attention blocks, with the JointAutoregressiveHierarchicalPriors
entropy path (context model + entropy parameters) of models/google.py.
Module trees and state_dict keys are the reference's.
"""
import torch.nn as nn

from ..layers import (AttentionBlock, ResidualBlock, ResidualBlockUpsample, ResidualBlockWithStride, Sequential,
                      conv3x3, subpel_conv3x3)
from .google import JointAutoregressiveHierarchicalPriors

__all__ = ["Cheng2020Anchor", "Cheng2020Attention"]


class Cheng2020Anchor(JointAutoregressiveHierarchicalPriors):
    """waseda.py:48-123."""

    # gradient buckets of g_a (compressai.distributed): g_a[4:], g_a[2:4], g_a[1], g_a[0] (the exposed last
    # bucket: ResidualBlockWithStride(3, N), 0.37 M parameters at N = 192)
    dp_tail_cuts = ("g_a.4", "g_a.2", "g_a.1")
    # g_s[4:] / g_s[:4] at N = 192: 17.5 / 29.5 MB of fp32 gradients
    dp_gs_cuts = ("g_s.4",)

    def __init__(self, N=192, channel=3, **kwargs):
        super().__init__(N=N, M=N, **kwargs)
        self.g_a = Sequential(
            ResidualBlockWithStride(channel, N, stride=2), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), ResidualBlock(N, N), conv3x3(N, N, stride=2))
        self.h_a = Sequential(
            conv3x3(N, N), nn.LeakyReLU(inplace=True), conv3x3(N, N), nn.LeakyReLU(inplace=True),
            conv3x3(N, N, stride=2), nn.LeakyReLU(inplace=True), conv3x3(N, N), nn.LeakyReLU(inplace=True),
            conv3x3(N, N, stride=2))
        self.h_s = Sequential(
            conv3x3(N, N), nn.LeakyReLU(inplace=True), subpel_conv3x3(N, N, 2), nn.LeakyReLU(inplace=True),
            conv3x3(N, N * 3 // 2), nn.LeakyReLU(inplace=True), subpel_conv3x3(N * 3 // 2, N * 3 // 2, 2),
            nn.LeakyReLU(inplace=True), conv3x3(N * 3 // 2, N * 2))
        self.g_s = Sequential(
            ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N),
            ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2),
            ResidualBlock(N, N), subpel_conv3x3(N, channel, 2))

    @classmethod
    def from_state_dict(cls, state_dict, channel=3):
        """waseda.py:115-121."""
        N = state_dict["g_a.0.conv1.weight"].size(0)
        net = cls(N, channel)
        net.load_state_dict(state_dict)
        return net


class Cheng2020Attention(Cheng2020Anchor):
    """waseda.py:126-158."""

    # g_a[5:] (10.0 MB of fp32 gradients at N = 192), g_a[2:5] (8.6 MB), g_a[1] (2.7 MB), g_a[0] (1.5 MB, exposed)
    dp_tail_cuts = ("g_a.5", "g_a.2", "g_a.1")
    # g_s[5:] (20.5 MB), g_s[:5] (32.6 MB); then the context model + entropy parameters (11.4 MB) and the hyper
    # path (31.2 MB): no bucket above 33 MB (the head was one 95.8 MB bucket).  Each phase boundary costs
    # ~25-35 us of split weight-gradient batches and reduce flushes: the fewest pieces
    # that keep every bucket under 40 MB
    dp_gs_cuts = ("g_s.5",)

    def __init__(self, N=192, channel=3, **kwargs):
        super().__init__(N=N, **kwargs)
        self.g_a = Sequential(
            ResidualBlockWithStride(channel, N, stride=2), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), AttentionBlock(N), ResidualBlock(N, N),
            ResidualBlockWithStride(N, N, stride=2), ResidualBlock(N, N), conv3x3(N, N, stride=2),
            AttentionBlock(N))
        self.g_s = Sequential(
            AttentionBlock(N), ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N),
            ResidualBlockUpsample(N, N, 2), AttentionBlock(N), ResidualBlock(N, N),
            ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N), subpel_conv3x3(N, channel, 2))
