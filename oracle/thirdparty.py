"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the third-party arithmetic the reference hot path calls but does not vendor:

* timm 0.4.5 ``PatchEmbed``, ``Block`` (``Attention`` + ``Mlp``)  — used at
  reference models/Compression/MCM.py:14, 300-302, 313-322, 339-348 and models/MAE/models_mae.py:17-55;
* compressai 1.2.4 ``EntropyBottleneck``, ``GaussianConditional``, ``LowerBound``, ``quantize_ste``,
  ``conv3x3``, ``subpel_conv3x3``, ``CompressionModel`` — used at MCM.py:8-12, 71-72, 115-162,
  741-744, 771-776 and utils/engine.py:79.

Neither package exists in this container, so these are restatements of the
published algorithms at the pinned versions; "parity unpinned" at this boundary as DESIGN.md says.
Parameter and buffer names match the upstream modules so reference state_dicts load unchanged.

Training-mode noise can be injected for reproducible comparisons: push tensors onto
``module.noise_queue``; when empty, ``uniform_(-0.5, 0.5)`` is used like upstream.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ------------------------------------------------------------------------------------ timm 0.4.5
def _pair(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


class PatchEmbed(nn.Module):
    """Image -> patch tokens: Conv2d(k=s=patch) then flatten(2).transpose(1, 2)."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.img_size = _pair(img_size)
        self.patch_size = _pair(patch_size)
        self.num_patches = (self.img_size[1] // self.patch_size[1]) * (self.img_size[0] // self.patch_size[0])
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=self.patch_size, stride=self.patch_size)

    def forward(self, x):
        _, _, h, w = x.shape
        assert h == self.img_size[0] and w == self.img_size[1], "Input image size doesn't match model"
        return self.proj(x).flatten(2).transpose(1, 2)


class Mlp(nn.Module):
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


class Attention(nn.Module):
    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.num_heads = num_heads
        self.scale = qk_scale or (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, x):
        b, n, c = x.shape
        qkv = self.qkv(x).reshape(b, n, 3, self.num_heads, c // self.num_heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        attn = ((q @ k.transpose(-2, -1)) * self.scale).softmax(dim=-1)
        x = (self.attn_drop(attn) @ v).transpose(1, 2).reshape(b, n, c)
        return self.proj_drop(self.proj(x))


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, qk_scale=None, drop=0.0, attn_drop=0.0,
                 drop_path=0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop,
                              proj_drop=drop)
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)

    def forward(self, x):
        x = x + self.drop_path(self.attn(self.norm1(x)))
        return x + self.drop_path(self.mlp(self.norm2(x)))


# ------------------------------------------------------------------------------ compressai 1.2.4
class LowerBound(nn.Module):
    def __init__(self, bound):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return torch.max(x, self.bound.to(x.dtype))


def quantize_ste(x):
    return (torch.round(x) - x).detach() + x


def conv3x3(in_ch, out_ch, stride=1):
    return nn.Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def subpel_conv3x3(in_ch, out_ch, r=1):
    return nn.Sequential(nn.Conv2d(in_ch, out_ch * r ** 2, kernel_size=3, padding=1), nn.PixelShuffle(r))


class EntropyModel(nn.Module):
    def __init__(self, likelihood_bound=1e-9, entropy_coder=None, entropy_coder_precision=16):
        super().__init__()
        self.entropy_coder_precision = int(entropy_coder_precision)
        self.use_likelihood_bound = likelihood_bound > 0
        if self.use_likelihood_bound:
            self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())
        self.noise_queue: list = []

    def quantize(self, inputs, mode, means=None):
        if mode == "noise":
            if self.noise_queue:
                noise = self.noise_queue.pop(0).to(inputs.dtype)
                assert noise.shape == inputs.shape, (noise.shape, inputs.shape)
            else:
                noise = torch.empty_like(inputs).uniform_(-0.5, 0.5)
            return inputs + noise
        outputs = inputs.clone()
        if means is not None:
            outputs -= means
        outputs = torch.round(outputs)
        if mode == "dequantize":
            if means is not None:
                outputs += means
            return outputs
        return outputs.int()

    def dequantize(self, inputs, means=None, dtype=torch.float):
        outputs = inputs.type(dtype) if means is None else inputs.type_as(means) + means
        return outputs


class EntropyBottleneck(EntropyModel):
    def __init__(self, channels, *args, tail_mass=1e-9, init_scale=10, filters=(3, 3, 3, 3), **kwargs):
        super().__init__(*args, **kwargs)
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        filters = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        for i in range(len(self.filters) + 1):
            init = np.log(np.expm1(1 / scale / filters[i + 1]))
            matrix = torch.Tensor(channels, filters[i + 1], filters[i])
            matrix.data.fill_(init)
            self.register_parameter(f"_matrix{i:d}", nn.Parameter(matrix))
            bias = torch.Tensor(channels, filters[i + 1], 1)
            nn.init.uniform_(bias, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(bias))
            if i < len(self.filters):
                factor = torch.Tensor(channels, filters[i + 1], 1)
                nn.init.zeros_(factor)
                self.register_parameter(f"_factor{i:d}", nn.Parameter(factor))
        self.quantiles = nn.Parameter(torch.Tensor(channels, 1, 3))
        init = torch.Tensor([-self.init_scale, 0, self.init_scale])
        self.quantiles.data = init.repeat(self.quantiles.size(0), 1, 1)
        target = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _get_medians(self):
        return self.quantiles[:, :, 1:2]

    def _logits_cumulative(self, inputs, stop_gradient):
        logits = inputs
        for i in range(len(self.filters) + 1):
            matrix = getattr(self, f"_matrix{i:d}")
            logits = torch.matmul(F.softplus(matrix.detach() if stop_gradient else matrix), logits)
            bias = getattr(self, f"_bias{i:d}")
            logits = logits + (bias.detach() if stop_gradient else bias)
            if i < len(self.filters):
                factor = getattr(self, f"_factor{i:d}")
                logits = logits + torch.tanh(factor.detach() if stop_gradient else factor) * torch.tanh(logits)
        return logits

    def _likelihood(self, inputs):
        lower = self._logits_cumulative(inputs - 0.5, stop_gradient=False)
        upper = self._logits_cumulative(inputs + 0.5, stop_gradient=False)
        sign = -torch.sign(lower + upper)
        sign = sign.detach()
        return torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))

    def loss(self):
        logits = self._logits_cumulative(self.quantiles, stop_gradient=True)
        return torch.abs(logits - self.target).sum()

    def forward(self, x, training=None):
        if training is None:
            training = self.training
        perm = np.arange(len(x.shape))
        perm[0], perm[1] = perm[1], perm[0]
        inv_perm = np.arange(len(x.shape))[np.argsort(perm)]
        x = x.permute(*perm).contiguous()
        shape = x.size()
        values = x.reshape(x.size(0), 1, -1)
        if training and self.noise_queue:
            # injected noise is given in the caller's NCHW layout
            n = self.noise_queue.pop(0).to(values.dtype).permute(*perm).contiguous().reshape(values.shape)
            self.noise_queue.insert(0, n)
        outputs = self.quantize(values, "noise" if training else "dequantize", self._get_medians())
        likelihood = self._likelihood(outputs)
        if self.use_likelihood_bound:
            likelihood = self.likelihood_lower_bound(likelihood)
        outputs = outputs.reshape(shape).permute(*inv_perm).contiguous()
        likelihood = likelihood.reshape(shape).permute(*inv_perm).contiguous()
        return outputs, likelihood


class GaussianConditional(EntropyModel):
    def __init__(self, scale_table, *args, scale_bound=0.11, tail_mass=1e-9, **kwargs):
        super().__init__(*args, **kwargs)
        self.tail_mass = float(tail_mass)
        self.register_buffer("scale_table", torch.Tensor(tuple(float(s) for s in scale_table)) if scale_table
                             else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]) if scale_bound is not None else None)
        self.lower_bound_scale = LowerBound(scale_bound)

    @staticmethod
    def _standardized_cumulative(inputs):
        return 0.5 * torch.erfc(float(-(2 ** -0.5)) * inputs)

    def _likelihood(self, inputs, scales, means=None):
        values = inputs - means if means is not None else inputs
        scales = self.lower_bound_scale(scales)
        values = torch.abs(values)
        upper = self._standardized_cumulative((0.5 - values) / scales)
        lower = self._standardized_cumulative((-0.5 - values) / scales)
        return upper - lower

    def forward(self, inputs, scales, means=None, training=None):
        if training is None:
            training = self.training
        outputs = self.quantize(inputs, "noise" if training else "dequantize", means)
        likelihood = self._likelihood(outputs, scales, means)
        if self.use_likelihood_bound:
            likelihood = self.likelihood_lower_bound(likelihood)
        return outputs, likelihood


class CompressionModel(nn.Module):
    def __init__(self, entropy_bottleneck_channels=None, init_weights=None):
        super().__init__()

    def aux_loss(self):
        return sum(m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck))


def get_scale_table(min_=0.11, max_=256, levels=64):
    return torch.exp(torch.linspace(math.log(min_), math.log(max_), levels))


# ------------------------------------------------------------------------------ pytorch_msssim
def _fspecial_gauss_1d(size, sigma, dtype=torch.float32):
    coords = torch.arange(size, dtype=torch.float) - size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    g /= g.sum()
    return g.to(dtype).unsqueeze(0).unsqueeze(0)


def _gaussian_filter(x, win):
    """win: [C, 1, 1, ws]; valid (no padding) separable filter along H then W."""
    c = x.shape[1]
    out = x
    for i, s in enumerate(x.shape[2:]):
        if s >= win.shape[-1]:
            out = F.conv2d(out, win.transpose(2 + i, -1), stride=1, padding=0, groups=c)
    return out


def ssim(x, y, data_range=1.0, win_size=11, win_sigma=1.5, K=(0.01, 0.03)):
    """pytorch_msssim.ssim (size_average=True), valid-padding separable gaussian window."""
    win = _fspecial_gauss_1d(win_size, win_sigma, x.dtype).unsqueeze(0).repeat(x.shape[1], 1, 1, 1)
    c1 = (K[0] * data_range) ** 2
    c2 = (K[1] * data_range) ** 2
    mu1, mu2 = _gaussian_filter(x, win), _gaussian_filter(y, win)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = _gaussian_filter(x * x, win) - mu1_sq
    s2 = _gaussian_filter(y * y, win) - mu2_sq
    s12 = _gaussian_filter(x * y, win) - mu1_mu2
    cs_map = (2 * s12 + c2) / (s1 + s2 + c2)
    ssim_map = ((2 * mu1_mu2 + c1) / (mu1_sq + mu2_sq + c1)) * cs_map
    return torch.flatten(ssim_map, 2).mean(-1).mean()


class SSIM(nn.Module):
    def __init__(self, data_range=255, size_average=True, win_size=11, win_sigma=1.5, channel=3, spatial_dims=2,
                 K=(0.01, 0.03), nonnegative_ssim=False):
        super().__init__()
        self.data_range, self.win_size, self.win_sigma, self.K = data_range, win_size, win_sigma, K

    def forward(self, x, y):
        return ssim(x, y, self.data_range, self.win_size, self.win_sigma, self.K)


def _ssim_per_channel(x, y, win, data_range, K=(0.01, 0.03)):
    c1 = (K[0] * data_range) ** 2
    c2 = (K[1] * data_range) ** 2
    mu1, mu2 = _gaussian_filter(x, win), _gaussian_filter(y, win)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = _gaussian_filter(x * x, win) - mu1_sq
    s2 = _gaussian_filter(y * y, win) - mu2_sq
    s12 = _gaussian_filter(x * y, win) - mu1_mu2
    cs_map = (2 * s12 + c2) / (s1 + s2 + c2)
    ssim_map = ((2 * mu1_mu2 + c1) / (mu1_sq + mu2_sq + c1)) * cs_map
    return torch.flatten(ssim_map, 2).mean(-1), torch.flatten(cs_map, 2).mean(-1)


def ms_ssim(x, y, data_range=255, win_size=11, win_sigma=1.5, weights=None, K=(0.01, 0.03)):
    """pytorch_msssim.ms_ssim (size_average=True; testing.py:48): five scales, relu'd per-channel cs / ssim,
    2x2 average pooling with padding H % 2, W % 2 between scales."""
    assert min(x.shape[-2:]) > (win_size - 1) * 2 ** 4
    w = torch.tensor(weights or [0.0448, 0.2856, 0.3001, 0.2363, 0.1333], dtype=x.dtype)
    win = _fspecial_gauss_1d(win_size, win_sigma, x.dtype).unsqueeze(0).repeat(x.shape[1], 1, 1, 1)
    mcs = []
    for i in range(w.numel()):
        s, cs = _ssim_per_channel(x, y, win, data_range, K)
        if i < w.numel() - 1:
            mcs.append(torch.relu(cs))
            pad = [d % 2 for d in x.shape[2:]]
            x = F.avg_pool2d(x, kernel_size=2, padding=pad)
            y = F.avg_pool2d(y, kernel_size=2, padding=pad)
    vals = torch.stack(mcs + [torch.relu(s)], dim=0)
    return torch.prod(vals ** w.view(-1, 1, 1), dim=0).mean()
