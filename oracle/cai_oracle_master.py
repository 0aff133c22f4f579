"""CPU oracle for the multi-modal (RGB + IR) codec: Master_compresser and
Guided_compresser (reference: compressai/models/master.py).

TEST INFRASTRUCTURE ONLY -- same rules as cai_oracle.py (only tests/, smoke()
and bench.py's cpu_baseline leg may use it).  Op-for-op fp32 restatement on CPU
torch; each class cites the master.py lines it follows.  timm is not
installed here: ``to_2tuple`` / ``DropPath`` (drop_path = 0 -> identity) and
``trunc_normal_`` (init only; parity runs copy weights by state_dict) are
restated inline.  Module names match the reference so state_dict keys agree.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import cai_oracle as O


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def conv1x1(cin, cout, stride=1):
    """master.py:21-23."""
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride)


def conv3x3(cin, cout, stride=1):
    """master.py:25-27."""
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1)


def conv(cin, cout, kernel_size=5, stride=2):
    """master.py:217-224."""
    return nn.Conv2d(cin, cout, kernel_size=kernel_size, stride=stride, padding=kernel_size // 2)


def deconv(cin, cout, kernel_size=5, stride=2):
    """master.py:87-95."""
    return nn.ConvTranspose2d(cin, cout, kernel_size=kernel_size, stride=stride, output_padding=stride - 1,
                              padding=kernel_size // 2)


ResidualBlock = O.ResidualBlock    # master.py:29-60 is layers.py:162-193 verbatim in behaviour


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
        return self.resblock3(self.resblock2(self.resblock1(out))) + out


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
        return self.deconv1(out + self.conv(x))


class Channel_aligner(nn.Module):
    """master.py:158-210: two weight-shared conv stacks, global average pools -> beta, gamma;
    out = gamma * feature2 + beta."""

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

    def _trunk(self, f):
        f = self.leaky_relu1(self.conv1(f))
        f = self.leaky_relu2(self.conv2(f))
        f = self.leaky_relu3(self.conv3(f))
        return self.leaky_relu4(self.conv4(f))

    def forward(self, feature1, feature2):
        beta = self.avgpool1(self.conv5(self._trunk(feature1)))
        gamma = self.avgpool2(self.conv6(self._trunk(feature2)))
        return gamma * feature2 + beta, beta, gamma


class PatchEmbed(nn.Module):
    """master.py:386-432 (norm_layer None)."""

    def __init__(self, img_size=(224, 224), patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        patch_size = _pair(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans, self.embed_dim = in_chans, embed_dim
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        B, C, H, W = x.shape
        assert H == self.img_size[0] and W == self.img_size[1]
        x = self.proj(x).flatten(2).transpose(1, 2)
        return self.norm(x) if self.norm is not None else x


def window_partition(x, ws):
    """master.py:435-445."""
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(-1, ws, ws, C)


def window_reverse(windows, ws, H, W):
    """master.py:448-462."""
    B = int(windows.shape[0] / (H * W / ws / ws))
    x = windows.view(B, H // ws, W // ws, ws, ws, -1)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(B, H, W, -1)


class Mlp(nn.Module):
    """master.py:465-482 (drop = 0)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        return self.drop(self.fc2(self.drop(self.act(self.fc1(x)))))


def relative_position_index(ws):
    """master.py:510-521: pair-wise relative position index inside a ws x ws window."""
    coords = torch.stack(torch.meshgrid([torch.arange(ws[0]), torch.arange(ws[1])], indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws[0] - 1
    rel[:, :, 1] += ws[1] - 1
    rel[:, :, 0] *= 2 * ws[1] - 1
    return rel.sum(-1)


class WindowAttention(nn.Module):
    """master.py:484-568: cross-attention, q from x (qkv1), k / v from guided (qkv2),
    relative position bias, optional shifted-window mask."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, window_size, num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window_size[0] - 1) * (2 * window_size[1] - 1), num_heads))
        self.register_buffer("relative_position_index", relative_position_index(window_size))
        self.qkv1 = nn.Linear(dim, dim, bias=qkv_bias)
        self.qkv2 = nn.Linear(dim, dim * 2, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x, guided, mask=None):
        B_, N, C = x.shape
        h = self.num_heads
        q = self.qkv1(x).reshape(B_, N, 1, h, C // h).permute(2, 0, 3, 1, 4)[0]
        kv = self.qkv2(guided).reshape(B_, N, 2, h, C // h).permute(2, 0, 3, 1, 4)
        k, v = kv[0], kv[1]
        attn = (q * self.scale) @ k.transpose(-2, -1)
        nn_ = self.window_size[0] * self.window_size[1]
        bias = self.relative_position_bias_table[self.relative_position_index.view(-1)].view(nn_, nn_, -1)
        attn = attn + bias.permute(2, 0, 1).contiguous().unsqueeze(0)
        if mask is not None:
            nW = mask.shape[0]
            attn = attn.view(B_ // nW, nW, h, N, N) + mask.unsqueeze(1).unsqueeze(0)
            attn = attn.view(-1, h, N, N)
        attn = self.attn_drop(self.softmax(attn))
        x = (attn @ v).transpose(1, 2).reshape(B_, N, C)
        return self.proj_drop(self.proj(x))


def shifted_window_mask(H, W, ws, shift):
    """master.py:620-640: -100 between tokens of different shifted-window regions."""
    img_mask = torch.zeros((1, H, W, 1))
    cnt = 0
    for hs in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for wsl in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img_mask[:, hs, wsl, :] = cnt
            cnt += 1
    mw = window_partition(img_mask, ws).view(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, float(-100.0)).masked_fill(m == 0, float(0.0))


class SwinTransformerBlock(nn.Module):
    """master.py:572-705 (drop_path = 0)."""

    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm,
                 fused_window_process=False):
        super().__init__()
        self.dim, self.input_resolution, self.num_heads = dim, input_resolution, num_heads
        self.window_size, self.shift_size, self.mlp_ratio = window_size, shift_size, mlp_ratio
        if min(self.input_resolution) <= self.window_size:
            self.shift_size = 0
            self.window_size = min(self.input_resolution)
        assert 0 <= self.shift_size < self.window_size
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=_pair(self.window_size), num_heads=num_heads, qkv_bias=qkv_bias,
                                    qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        attn_mask = (shifted_window_mask(*self.input_resolution, self.window_size, self.shift_size)
                     if self.shift_size > 0 else None)
        self.register_buffer("attn_mask", attn_mask)
        self.fused_window_process = fused_window_process

    def forward(self, x, guided):
        H, W = self.input_resolution
        B, L, C = x.shape
        assert L == H * W
        ws, sh = self.window_size, self.shift_size
        shortcut = x
        x = self.norm1(x).view(B, H, W, C)
        guided = self.norm1(guided).view(B, H, W, C)
        if sh > 0:
            x = torch.roll(x, shifts=(-sh, -sh), dims=(1, 2))
            guided = torch.roll(guided, shifts=(-sh, -sh), dims=(1, 2))
        xw = window_partition(x, ws).view(-1, ws * ws, C)
        gw = window_partition(guided, ws).view(-1, ws * ws, C)
        aw = self.attn(xw, gw, mask=self.attn_mask).view(-1, ws, ws, C)
        x = window_reverse(aw, ws, H, W)
        if sh > 0:
            x = torch.roll(x, shifts=(sh, sh), dims=(1, 2))
        x = shortcut + x.view(B, H * W, C)
        return x + self.mlp(self.norm2(x))


class Spatial_aligner(nn.Module):
    """master.py:708-742: patch embeddings of x and guided, two (shifted) cross-attention
    Swin blocks, then the (B, L, C) tokens re-read as (B, C, H/2, W/2) -- a view, not a
    permute, exactly as the reference -- and a k2 s2 transposed conv."""

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
        self.recovery = nn.ConvTranspose2d(96, out_channel, kernel_size=2, stride=2)

    def forward(self, x, guided):
        B, C, H, W = x.shape
        out = self.patch_embeding1(x)
        g = self.patch_embeding2(guided)
        for layer in self.blocks:
            out = layer(out, g)
        out = out.contiguous().view(B, self.embed_dim, H // 2, W // 2)
        return self.recovery(out)


class Master_decoder(nn.Module):
    """master.py:745-811."""

    def __init__(self, N=192, M=192, channel=64 * 2, width=224, height=224, first_stride=2, master_chl=3):
        super().__init__()
        self.encoder_first_stride = first_stride
        width //= first_stride
        height //= first_stride
        self.g_s_conv1 = deconv(M, N, kernel_size=5, stride=2)
        self.g_s_gdn1 = O.GDN(N, inverse=True)
        self.sp_aligner1 = Spatial_aligner(input_resolution=(width // 4, height // 4))
        self.g_s_conv2 = deconv(2 * N, N, kernel_size=5, stride=2)
        self.g_s_gdn2 = O.GDN(N, inverse=True)
        self.sp_aligner2 = Spatial_aligner(input_resolution=(width // 2, height // 2))
        self.g_s_conv3 = deconv(2 * N, N, kernel_size=5, stride=2)
        self.g_s_gdn3 = O.GDN(N, inverse=True)
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
        o = torch.cat([self.sp_aligner1(o, g1), o], dim=1)
        o = self.g_s_gdn2(self.g_s_conv2(o))
        o = torch.cat([self.sp_aligner2(o, g2), o], dim=1)
        o = self.g_s_gdn3(self.g_s_conv3(o))
        o = torch.cat([self.sp_aligner3(o, g3), o], dim=1)
        return {"x_feature_hat": self.g_s_conv4(o)}


def _jahp_tail(model, N, M):
    """The hyperprior + context entropy path shared by Master/Guided (master.py:240-270, 1231-1265)."""
    model.h_a = nn.Sequential(conv(M, N, stride=1, kernel_size=3), nn.LeakyReLU(inplace=True),
                              conv(N, N, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                              conv(N, N, stride=2, kernel_size=5))
    model.h_s = nn.Sequential(deconv(N, M, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                              deconv(M, M * 3 // 2, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                              conv(M * 3 // 2, M * 2, stride=1, kernel_size=3))
    model.entropy_parameters = nn.Sequential(
        nn.Conv2d(M * 12 // 3, M * 10 // 3, 1), nn.LeakyReLU(inplace=True),
        nn.Conv2d(M * 10 // 3, M * 8 // 3, 1), nn.LeakyReLU(inplace=True),
        nn.Conv2d(M * 8 // 3, M * 6 // 3, 1))
    model.context_prediction = O.MaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)
    model.gaussian_conditional = O.GaussianConditional(None)
    model.N, model.M = int(N), int(M)


def _entropy(model, y):
    z = model.h_a(y)
    z_hat, z_lik = model.entropy_bottleneck(z)
    params = model.h_s(z_hat)
    y_hat = model.gaussian_conditional.quantize(y, "noise" if model.training else "dequantize")
    ctx = model.context_prediction(y_hat)
    scales_hat, means_hat = model.entropy_parameters(torch.cat((params, ctx), dim=1)).chunk(2, 1)
    _, y_lik = model.gaussian_conditional(y, scales_hat, means=means_hat)
    return y_hat, y_lik, z_lik


class Master_compresser(O.MeanScaleHyperprior):
    """master.py:837-951."""

    def __init__(self, width=256, height=256, channel=3, N=192, M=192):
        super().__init__(M, M)
        master_chl, guided_chl, master_stride, guided_stride = 3, 1, 2, 1
        if channel == 1:
            master_chl, guided_chl, guided_stride, master_stride = 1, 3, 2, 1
        self.fencoder1 = Feature_encoder(in_channel=master_chl, out_channel=64, stride=master_stride)
        self.fencoder2 = Feature_encoder(in_channel=guided_chl, out_channel=64, stride=guided_stride)
        self.ch_aligner = Channel_aligner()
        self.g_a = nn.Sequential(conv(64 * 2, N), O.GDN(N), conv(N, N), O.GDN(N), conv(N, N), O.GDN(N), conv(N, M))
        _jahp_tail(self, N, M)
        self.decoder = Master_decoder(N=192, M=192, channel=64 * 2, width=width, height=height, first_stride=2,
                                      master_chl=master_chl)
        self.fdecoder = Feature_decoder(in_channel=64 * 3, out_channel=master_chl, stride=master_stride)

    def forward(self, x, guided_hat, guided_hidden):
        x_feature = self.fencoder1(x)
        guided_feature = self.fencoder2(guided_hat)
        guided_align, beta, gamma = self.ch_aligner(x_feature, guided_feature)
        y = self.g_a(torch.cat([x_feature, guided_align], dim=1))
        y_hat, y_lik, z_lik = _entropy(self, y)
        res = self.decoder(y_hat, guided_hidden)
        out = self.fdecoder(torch.cat([res["x_feature_hat"], guided_align], dim=1))
        return {"x_hat": out, "likelihoods": {"y": y_lik, "z": z_lik}}


class Encoder1(nn.Module):
    """master.py:1167-1189."""

    def __init__(self, N, M, channel=1, first_stride=2, **kwargs):
        super().__init__()
        self.g_a_conv1 = conv(channel, N, kernel_size=5, stride=first_stride)
        self.g_a_gdn1 = O.GDN(N)
        self.g_a_conv2 = conv(N, N)
        self.g_a_gdn2 = O.GDN(N)
        self.g_a_conv3 = conv(N, N)
        self.g_a_gdn3 = O.GDN(N)
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
        self.g_s_gdn1 = O.GDN(N, inverse=True)
        self.g_s_conv2 = deconv(N, N)
        self.g_s_gdn2 = O.GDN(N, inverse=True)
        self.g_s_conv3 = deconv(N, N)
        self.g_s_gdn3 = O.GDN(N, inverse=True)
        self.g_s_conv4 = deconv(N, channel, kernel_size=5, stride=first_stride)

    def forward(self, y_hat):
        g1 = self.g_s_gdn1(self.g_s_conv1(y_hat))
        g2 = self.g_s_gdn2(self.g_s_conv2(g1))
        g3 = self.g_s_gdn3(self.g_s_conv3(g2))
        return self.g_s_conv4(g3), g1, g2, g3


class Guided_compresser(O.MeanScaleHyperprior):
    """master.py:1215-1295."""

    def __init__(self, N=192, M=192, channel=1, first_stride=2, **kwargs):
        super().__init__(N=N, M=M, **kwargs)
        self.first_stride = first_stride
        self.enc1 = Encoder1(N, M, channel, first_stride)
        self.dec1 = Decoder1(N, M, channel, first_stride)
        _jahp_tail(self, N, M)

    def forward(self, x):
        y1, ga1, ga2, ga3 = self.enc1(x)
        y1_hat, y_lik, z_lik = _entropy(self, y1)
        x1_hat, gs1, gs2, gs3 = self.dec1(y1_hat)
        return {"x_hat": x1_hat, "likelihoods": {"y": y_lik, "z": z_lik},
                "hidden": {"ga1": ga1, "ga2": ga2, "ga3": ga3, "gs1": gs1, "gs2": gs2, "gs3": gs3}}
