"""Multi-modal (RGB + IR) codec of the reference fork (compressai/models/master.py).

Guided_compresser codes the guide modality and exposes its analysis /
synthesis activations ("hidden"); Master_compresser codes the other modality
with (a) feature encoders + a Channel_aligner (global affine alignment of the
guide features) before its analysis transform and (b) Spatial_aligners
(shifted-window cross-attention Swin blocks, queries from the master, keys /
values from the guide's synthesis activations) between its synthesis layers.

Module trees, names and state_dict keys follow the reference; everything runs
on the HIP kernels: convs (csrc/conv.hip), GDN, residual / cat glue
(csrc/elementwise.hip), LayerNorm / GELU / window attention / channel pooling
(csrc/swin.hip).  Token sequences (B, L, C) are pixel-major [B, C, H', W']
tensors, i.e. the reference's flattened token order.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .._native import ACT_LEAKY, ACT_NONE, MASK_LEAKY
from .._ops import (AddActFn, CatFn, ChannelAffineFn, ChannelMeanFn, ConvFn, ConvSpec, GeluFn, LayerNormFn,
                    WindowAttnFn)
from ..entropy_models import GaussianConditional
from ..layers import GDN, MaskedConv2d, ResidualBlock, Sequential
from ..layers.conv import Conv2d, ConvTranspose2d
from .._prepack import prepacked_forward
from .google import MeanScaleHyperprior, _ARCoding

__all__ = ["Master_compresser", "Guided_compresser", "Spatial_aligner", "Channel_aligner", "SwinTransformerBlock",
           "WindowAttention", "Feature_encoder", "Feature_decoder", "Master_decoder", "Encoder1", "Decoder1"]

_SLOPE = 0.01


def conv1x1(cin, cout, stride=1):
    """master.py:21-23."""
    return Conv2d(cin, cout, kernel_size=1, stride=stride)


def conv3x3(cin, cout, stride=1):
    """master.py:25-27."""
    return Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1)


def conv(cin, cout, kernel_size=5, stride=2):
    """master.py:217-224."""
    return Conv2d(cin, cout, kernel_size=kernel_size, stride=stride, padding=kernel_size // 2)


def deconv(cin, cout, kernel_size=5, stride=2):
    """master.py:87-95."""
    return ConvTranspose2d(cin, cout, kernel_size=kernel_size, stride=stride, output_padding=stride - 1,
                           padding=kernel_size // 2)


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


# ---------------------------------------------------------------------------
# token-wise layers
# ---------------------------------------------------------------------------

_LINEAR_SPEC = ConvSpec(1, 1, 0)


class Linear(nn.Linear):
    """nn.Linear on pixel-major tokens: a 1x1 conv on the implicit-GEMM kernels (weight viewed [out, in, 1, 1])."""

    def forward(self, x):
        w = self.weight.view(self.out_features, self.in_features, 1, 1)
        return ConvFn.apply(x, w, self.bias, _LINEAR_SPEC)


class LayerNorm(nn.LayerNorm):
    def forward(self, x):
        return LayerNormFn.apply(x, self.weight, self.bias, float(self.eps))


class GELU(nn.GELU):
    def forward(self, x):
        return GeluFn.apply(x)


class Mlp(nn.Module):
    """master.py:465-482 (drop = 0)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


def _relative_position_index(ws):
    coords = torch.stack(torch.meshgrid([torch.arange(ws[0]), torch.arange(ws[1])], indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws[0] - 1
    rel[:, :, 1] += ws[1] - 1
    rel[:, :, 0] *= 2 * ws[1] - 1
    return rel.sum(-1)


class WindowAttention(nn.Module):
    """master.py:484-568.  The attention core runs in cai_window_attn_{fwd,bwd}; proj is a Linear."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, window_size, num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window_size[0] - 1) * (2 * window_size[1] - 1), num_heads))
        idx = _relative_position_index(window_size)
        self.register_buffer("relative_position_index", idx)
        self.register_buffer("_rel_index_i32", idx.to(torch.int32).contiguous(), persistent=False)
        self.qkv1 = Linear(dim, dim, bias=qkv_bias)
        self.qkv2 = Linear(dim, dim * 2, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        self.softmax = nn.Softmax(dim=-1)

    def attend(self, xn, gn, Hr, Wr, shift, mask):
        q = self.qkv1(xn)
        kv = self.qkv2(gn)
        cfg = (Hr, Wr, self.num_heads, self.window_size[0], shift, float(self.scale))
        return self.proj(WindowAttnFn.apply(q, kv, self.relative_position_bias_table, self._rel_index_i32, mask,
                                            cfg))


def _shifted_window_mask(H, W, ws, shift):
    """master.py:620-640."""
    img_mask = torch.zeros((1, H, W, 1))
    cnt = 0
    for hs in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for wsl in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img_mask[:, hs, wsl, :] = cnt
            cnt += 1
    mw = img_mask.view(1, H // ws, ws, W // ws, ws, 1).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, float(-100.0)).masked_fill(m == 0, float(0.0))


class SwinTransformerBlock(nn.Module):
    """master.py:572-705: cross-attention Swin block (drop_path 0), tokens pixel-major."""

    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=GELU, norm_layer=LayerNorm,
                 fused_window_process=False):
        super().__init__()
        self.dim, self.input_resolution, self.num_heads = dim, input_resolution, num_heads
        self.window_size, self.shift_size, self.mlp_ratio = window_size, shift_size, mlp_ratio
        if min(self.input_resolution) <= self.window_size:
            self.shift_size = 0
            self.window_size = min(self.input_resolution)
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=_pair(self.window_size), num_heads=num_heads, qkv_bias=qkv_bias,
                                    qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        mask = (_shifted_window_mask(*self.input_resolution, self.window_size, self.shift_size)
                if self.shift_size > 0 else None)
        self.register_buffer("attn_mask", mask)
        self.fused_window_process = fused_window_process

    def forward(self, x, guided):
        H, W = self.input_resolution
        if x.shape[2] * x.shape[3] != H * W:
            raise ValueError("input feature has wrong size")
        a = self.attn.attend(self.norm1(x), self.norm1(guided), H, W, self.shift_size, self.attn_mask)
        x = AddActFn.apply(x, a, ACT_NONE, 0.0)
        return AddActFn.apply(x, self.mlp(self.norm2(x)), ACT_NONE, 0.0)


class PatchEmbed(nn.Module):
    """master.py:386-432 (norm None): a k=s=patch conv; its pixel-major output IS the token sequence."""

    def __init__(self, img_size=(224, 224), patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        patch_size = _pair(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans, self.embed_dim = in_chans, embed_dim
        self.proj = Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        B, C, H, W = x.shape
        if H != self.img_size[0] or W != self.img_size[1]:
            raise ValueError(f"Input image size ({H}*{W}) doesn't match model ({self.img_size[0]}*{self.img_size[1]}).")
        x = self.proj(x)
        return self.norm(x) if self.norm is not None else x


class Spatial_aligner(nn.Module):
    """master.py:708-742."""

    def __init__(self, in_channel=192, out_channel=192, input_resolution=(224, 224)):
        super().__init__()
        self.window_size, self.patch_size = 4, 2
        self.input_resolution = input_resolution
        self.embed_dim = 96
        self.patch_embeding1 = PatchEmbed(img_size=input_resolution, patch_size=2, in_chans=in_channel, embed_dim=96)
        self.patch_embeding2 = PatchEmbed(img_size=input_resolution, patch_size=2, in_chans=in_channel, embed_dim=96)
        res = (input_resolution[0] // 2, input_resolution[1] // 2)
        self.blocks = nn.ModuleList([SwinTransformerBlock(dim=96, num_heads=3, window_size=4, input_resolution=res,
                                                          shift_size=0 if i % 2 == 0 else 2) for i in range(2)])
        self.recovery = ConvTranspose2d(96, out_channel, kernel_size=2, stride=2)

    def forward(self, x, guided):
        B, C, H, W = x.shape
        out = self.patch_embeding1(x)
        g = self.patch_embeding2(guided)
        for layer in self.blocks:
            out = layer(out, g)
        # master.py:738: the (B, L, C) tokens are re-read as (B, C, H/2, W/2) -- a view of the
        # token memory, not a permute; the pixel-major token tensor is that memory
        tokens = out.permute(0, 2, 3, 1)
        if not tokens.is_contiguous():
            tokens = tokens.contiguous()
        return self.recovery(tokens.reshape(B, self.embed_dim, H // 2, W // 2))


# ---------------------------------------------------------------------------
# feature encoder / decoder, channel aligner
# ---------------------------------------------------------------------------

class Feature_encoder(nn.Module):
    """master.py:68-84."""

    def __init__(self, in_channel=3, out_channel=64, stride=1):
        super().__init__()
        self.conv1 = conv3x3(in_channel, out_channel, stride)
        self.resblock1 = ResidualBlock(64, 64)
        self.resblock2 = ResidualBlock(64, 64)
        self.resblock3 = ResidualBlock(64, 64)

    def forward(self, x):
        out = self.conv1(x)
        r = self.resblock3(self.resblock2(self.resblock1(out)))
        return AddActFn.apply(r, out, ACT_NONE, 0.0)


class Feature_decoder(nn.Module):
    """master.py:99-118."""

    def __init__(self, in_channel=64 * 3, out_channel=3, stride=1):
        super().__init__()
        self.resblock1 = ResidualBlock(in_channel, 64)
        self.resblock2 = ResidualBlock(64, 64)
        self.resblock3 = ResidualBlock(64, 64)
        self.deconv1 = deconv(64, out_channel, kernel_size=3, stride=stride)
        self.conv = conv1x1(in_channel, 64)

    def forward(self, x):
        out = self.resblock3(self.resblock2(self.resblock1(x)))
        return self.deconv1(AddActFn.apply(out, self.conv(x), ACT_NONE, 0.0))


class Channel_aligner(nn.Module):
    """master.py:158-210: weight-shared 4-conv trunks, conv5 / conv6 heads, global average
    pools -> beta / gamma, out = gamma * feature2 + beta."""

    def __init__(self):
        super().__init__()
        self.conv1 = conv3x3(64, 256)
        self.leaky_relu1 = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(256, 256)
        self.leaky_relu2 = nn.LeakyReLU(inplace=True)
        self.conv3 = conv3x3(256, 256)
        self.leaky_relu3 = nn.LeakyReLU(inplace=True)
        self.conv4 = conv3x3(256, 256)
        self.leaky_relu4 = nn.LeakyReLU(inplace=True)
        self.conv5 = conv3x3(256, 64)
        self.conv6 = conv3x3(256, 64)
        self.avgpool1 = nn.AdaptiveAvgPool2d(1)
        self.avgpool2 = nn.AdaptiveAvgPool2d(1)

    def _branch(self, f, head):
        kw = dict(act=ACT_LEAKY, act_param=_SLOPE, act_bwd_downstream=True)
        m = dict(in_mask=MASK_LEAKY, in_mask_param=_SLOPE)
        f = self.conv1.run(f, **kw)
        f = self.conv2.run(f, **kw, **m)
        f = self.conv3.run(f, **kw, **m)
        f = self.conv4.run(f, **kw, **m)
        return ChannelMeanFn.apply(head.run(f, **m))

    def forward(self, feature1, feature2):
        beta = self._branch(feature1, self.conv5)
        gamma = self._branch(feature2, self.conv6)
        return ChannelAffineFn.apply(feature2, gamma, beta), beta, gamma


class Master_decoder(nn.Module):
    """master.py:745-811."""

    def __init__(self, N=192, M=192, channel=64 * 2, width=224, height=224, first_stride=2, master_chl=3):
        super().__init__()
        self.encoder_first_stride = first_stride
        width //= first_stride
        height //= first_stride
        self.g_s_conv1 = deconv(M, N, kernel_size=5, stride=2)
        self.g_s_gdn1 = GDN(N, inverse=True)
        self.sp_aligner1 = Spatial_aligner(input_resolution=(width // 4, height // 4))
        self.g_s_conv2 = deconv(2 * N, N, kernel_size=5, stride=2)
        self.g_s_gdn2 = GDN(N, inverse=True)
        self.sp_aligner2 = Spatial_aligner(input_resolution=(width // 2, height // 2))
        self.g_s_conv3 = deconv(2 * N, N, kernel_size=5, stride=2)
        self.g_s_gdn3 = GDN(N, inverse=True)
        self.sp_aligner3 = Spatial_aligner(input_resolution=(width, height))
        self.g_s_conv4 = deconv(2 * N, channel, kernel_size=5, stride=first_stride)
        self.master_chl = master_chl
        if master_chl == 1:
            self.downsample1 = conv(N, N, kernel_size=5, stride=2)
            self.downsample2 = conv(N, N, kernel_size=5, stride=2)
            self.downsample3 = conv(N, N, kernel_size=5, stride=2)

    def forward(self, x, guide_hidden):
        g1, g2, g3 = guide_hidden["gs1"], guide_hidden["gs2"], guide_hidden["gs3"]
        if self.master_chl == 1:
            g1, g2, g3 = self.downsample1(g1), self.downsample2(g2), self.downsample3(g3)
        o = self.g_s_gdn1(self.g_s_conv1(x))
        o = CatFn.apply(self.sp_aligner1(o, g1), o)
        o = self.g_s_gdn2(self.g_s_conv2(o))
        o = CatFn.apply(self.sp_aligner2(o, g2), o)
        o = self.g_s_gdn3(self.g_s_conv3(o))
        o = CatFn.apply(self.sp_aligner3(o, g3), o)
        return {"x_feature_hat": self.g_s_conv4(o)}


# ---------------------------------------------------------------------------
# codecs
# ---------------------------------------------------------------------------

def _jahp_tail(model, N, M):
    """Hyperprior + context entropy path shared by Master / Guided (master.py:240-270, 1231-1265)."""
    model.h_a = Sequential(conv(M, N, stride=1, kernel_size=3), nn.LeakyReLU(inplace=True),
                           conv(N, N, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                           conv(N, N, stride=2, kernel_size=5))
    model.h_s = Sequential(deconv(N, M, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                           deconv(M, M * 3 // 2, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                           conv(M * 3 // 2, M * 2, stride=1, kernel_size=3))
    model.entropy_parameters = Sequential(
        Conv2d(M * 12 // 3, M * 10 // 3, 1), nn.LeakyReLU(inplace=True),
        Conv2d(M * 10 // 3, M * 8 // 3, 1), nn.LeakyReLU(inplace=True),
        Conv2d(M * 8 // 3, M * 6 // 3, 1))
    model.context_prediction = MaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)
    model.gaussian_conditional = GaussianConditional(None)
    model.N, model.M = int(N), int(M)


def _entropy(model, y):
    z = model.h_a(y)
    z_hat, z_lik = model.entropy_bottleneck(z)
    params = model._dp_mark("params", model.h_s(z_hat))
    yq = model._dp_mark("yq", y)        # y as quantize / the GaussianConditional read it (Master's dp_phases)
    y_hat = model.gaussian_conditional.quantize(yq, "noise" if model.training else "dequantize")
    ctx = model.context_prediction(y_hat)
    scales_hat, means_hat = model.entropy_parameters(CatFn.apply(params, ctx)).chunk(2, 1)
    _, y_lik = model.gaussian_conditional(yq, scales_hat, means=means_hat)
    return y_hat, y_lik, z_lik


class Master_compresser(_ARCoding, MeanScaleHyperprior):
    """master.py:837-951: net(x, guided_hat, guided_hidden) -> {"x_hat", "likelihoods"}."""

    # data parallelism: the feature encoders + channel aligner are the tail (guided_align also feeds fdecoder,
    # so the cut is {x_feature, guided_align}, not g_a's output); the inherited g_s is never used (its
    # gradients stay zero, as in the reference, master.py:839)
    dp_tail = ("fencoder1.", "fencoder2.", "ch_aligner.")
    dp_tail_cuts = ()     # one tail bucket (10.6 MB against a ~57 ms pair step)

    def __init__(self, width=256, height=256, channel=3, N=192, M=192):
        super().__init__(M, M)
        master_chl, guided_chl, master_stride, guided_stride = 3, 1, 2, 1
        if channel == 1:
            master_chl, guided_chl, guided_stride, master_stride = 1, 3, 2, 1
        self.fencoder1 = Feature_encoder(in_channel=master_chl, out_channel=64, stride=master_stride)
        self.fencoder2 = Feature_encoder(in_channel=guided_chl, out_channel=64, stride=guided_stride)
        self.ch_aligner = Channel_aligner()
        self.g_a = Sequential(conv(64 * 2, N), GDN(N), conv(N, N), GDN(N), conv(N, N), GDN(N), conv(N, M))
        _jahp_tail(self, N, M)
        self.decoder = Master_decoder(N=192, M=192, channel=64 * 2, width=width, height=height, first_stride=2,
                                      master_chl=master_chl)
        self.fdecoder = Feature_decoder(in_channel=64 * 3, out_channel=master_chl, stride=master_stride)

    def dp_phases(self):
        """Gradient buckets in backward order (compressai.distributed): the synthesis (decoder + fdecoder), the
        context model + entropy parameters, the hyper path, g_a, then the tail.  guided_align feeds both g_a
        and fdecoder: its fdecoder branch is a cut of its own ("ga_fd"), so the synthesis phase stops there
        and the g_a phase carries that gradient on to the tail cut.  g_a's output y is read by the hyper path
        and (as "yq") by quantize / the GaussianConditional: the context phase stops at "yq", not at y, which
        the hyper path below its "params" cut also reaches."""
        return [(["decoder.", "fdecoder."], ["loss"], ["gs_in", "lik_y", "lik_z", "ga_fd"]),
                (["entropy_parameters.", "context_prediction."], ["gs_in", "lik_y"], ["params", "yq"]),
                (None, ["params", "lik_z"], ["ga_out"]),
                (["g_a."], ["ga_out", "yq", "ga_fd"], ["y"]),
                (list(self.dp_tail), ["y"], [])]

    def forward(self, x, guided_hat, guided_hidden):
        x_feature = self.fencoder1(x)
        guided_feature = self.fencoder2(guided_hat)
        guided_align, beta, gamma = self.ch_aligner(x_feature, guided_feature)
        x_feature, guided_align = self._dp_cut(x_feature, guided_align)
        y = self._dp_mark("ga_out", self.g_a(CatFn.apply(x_feature, guided_align)))
        y_hat, y_lik, z_lik = _entropy(self, y)
        res = self.decoder(self._dp_mark("gs_in", y_hat), guided_hidden)
        out = self.fdecoder(CatFn.apply(res["x_feature_hat"], self._dp_mark("ga_fd", guided_align)))
        return {"x_hat": out, "likelihoods": {"y": self._dp_mark("lik_y", y_lik), "z": self._dp_mark("lik_z", z_lik)}}

    @torch.no_grad()
    def compress(self, x, guided_hat):
        """master.py:953-991: the channel-aligner's beta / gamma travel as side information."""
        with prepacked_forward(self):
            x_feature = self.fencoder1(x)
            guided_feature = self.fencoder2(guided_hat)
            guided_align, beta, gamma = self.ch_aligner(x_feature, guided_feature)
            y = self.g_a(CatFn.apply(x_feature, guided_align))
            z = self.h_a(y)
            z_strings = self.entropy_bottleneck.compress(z)
            z_hat = self.entropy_bottleneck.decompress(z_strings, z.size()[-2:])
            params = self.h_s(z_hat)
            y_strings = self._ar_encode_all(y, params)
        return {"strings": [y_strings, z_strings], "shape": z.size()[-2:], "gamma": gamma, "beta": beta}

    @torch.no_grad()
    def decompress(self, out_net, out_net_guided):
        """master.py:1054-1107: the guide's decoded image and synthesis activations condition the decoder."""
        strings, shape, beta, gamma = out_net["strings"], out_net["shape"], out_net["beta"], out_net["gamma"]
        assert isinstance(strings, list) and len(strings) == 2
        self._warn_gpu(self)
        with prepacked_forward(self):
            guided_align = ChannelAffineFn.apply(self.fencoder2(out_net_guided["x_hat"]), gamma, beta)
            z_hat = self.entropy_bottleneck.decompress(strings[1], shape)
            params = self.h_s(z_hat)
            y_hat = self._ar_decode_all(strings[0], params)
            res = self.decoder(y_hat, out_net_guided["hidden"])
            x_hat = self.fdecoder(CatFn.apply(res["x_feature_hat"], guided_align)).clamp_(0, 1)
        return {"x_hat": x_hat}


class Encoder1(nn.Module):
    """master.py:1167-1189."""

    def __init__(self, N, M, channel=1, first_stride=2, **kwargs):
        super().__init__()
        self.g_a_conv1 = conv(channel, N, kernel_size=5, stride=first_stride)
        self.g_a_gdn1 = GDN(N)
        self.g_a_conv2 = conv(N, N)
        self.g_a_gdn2 = GDN(N)
        self.g_a_conv3 = conv(N, N)
        self.g_a_gdn3 = GDN(N)
        self.g_a_conv4 = conv(N, M)

    def forward(self, x):
        g1 = self.g_a_gdn1(self.g_a_conv1(x))
        g2 = self.g_a_gdn2(self.g_a_conv2(g1))
        g3 = self.g_a_gdn3(self.g_a_conv3(g2))
        return self.g_a_conv4(g3), g1, g2, g3


class Decoder1(nn.Module):
    """master.py:1192-1212."""

    def __init__(self, N, M, channel=1, first_stride=2, **kwargs):
        super().__init__()
        self.g_s_conv1 = deconv(M, N)
        self.g_s_gdn1 = GDN(N, inverse=True)
        self.g_s_conv2 = deconv(N, N)
        self.g_s_gdn2 = GDN(N, inverse=True)
        self.g_s_conv3 = deconv(N, N)
        self.g_s_gdn3 = GDN(N, inverse=True)
        self.g_s_conv4 = deconv(N, channel, kernel_size=5, stride=first_stride)

    def forward(self, y_hat):
        g1 = self.g_s_gdn1(self.g_s_conv1(y_hat))
        g2 = self.g_s_gdn2(self.g_s_conv2(g1))
        g3 = self.g_s_gdn3(self.g_s_conv3(g2))
        return self.g_s_conv4(g3), g1, g2, g3


class Guided_compresser(_ARCoding, MeanScaleHyperprior):
    """master.py:1215-1295: net(x) -> {"x_hat", "likelihoods", "hidden": {ga1..3, gs1..3}}."""

    def __init__(self, N=192, M=192, channel=1, first_stride=2, **kwargs):
        super().__init__(N=N, M=M, **kwargs)
        self.first_stride = first_stride
        self.enc1 = Encoder1(N, M, channel, first_stride)
        self.dec1 = Decoder1(N, M, channel, first_stride)
        _jahp_tail(self, N, M)

    @property
    def downsampling_factor(self) -> int:
        return 2 ** (4 + 2)

    def forward(self, x):
        y1, ga1, ga2, ga3 = self.enc1(x)
        y1_hat, y_lik, z_lik = _entropy(self, y1)
        x1_hat, gs1, gs2, gs3 = self.dec1(y1_hat)
        return {"x_hat": x1_hat, "likelihoods": {"y": y_lik, "z": z_lik},
                "hidden": {"ga1": ga1, "ga2": ga2, "ga3": ga3, "gs1": gs1, "gs2": gs2, "gs3": gs3}}

    @torch.no_grad()
    def compress(self, x):
        """master.py:1297-1335."""
        self._warn_gpu(self)
        with prepacked_forward(self):
            y, ga1, ga2, ga3 = self.enc1(x)
            z = self.h_a(y)
            z_strings = self.entropy_bottleneck.compress(z)
            z_hat = self.entropy_bottleneck.decompress(z_strings, z.size()[-2:])
            params = self.h_s(z_hat)
            y_strings = self._ar_encode_all(y, params)
        return {"strings": [y_strings, z_strings], "shape": z.size()[-2:],
                "hidden": {"ga1": ga1, "ga2": ga2, "ga3": ga3}}

    @torch.no_grad()
    def decompress(self, strings, shape):
        """master.py:1381-1424: the reconstruction and the synthesis activations the Master codec needs."""
        assert isinstance(strings, list) and len(strings) == 2
        self._warn_gpu(self)
        with prepacked_forward(self):
            z_hat = self.entropy_bottleneck.decompress(strings[1], shape)
            params = self.h_s(z_hat)
            y_hat = self._ar_decode_all(strings[0], params)
            x_hat, gs1, gs2, gs3 = self.dec1(y_hat)
        return {"x_hat": x_hat.clamp(0, 1), "hidden": {"gs1": gs1, "gs2": gs2, "gs3": gs3}}
