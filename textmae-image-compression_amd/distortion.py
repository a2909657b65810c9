"""Distortion terms of MCM.forward_loss (reference MCM.py:690-712).

Not part of the measured encode + rate + decode path (SURVEY.md §8d reports it separately); these
run as device-side torch ops on the reconstruction.  SSIM follows pytorch_msssim (unpinned in
the reference's requirements): 11-tap gaussian window, sigma 1.5, valid padding, K = (0.01, 0.03),
data_range 1, mean over channels and batch.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

_WIN = {}


def _window(size, sigma, channels, dtype, device):
    key = (size, sigma, channels, dtype, device)
    if key not in _WIN:
        coords = torch.arange(size, dtype=torch.float) - size // 2
        g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
        g = (g / g.sum()).to(dtype)
        _WIN[key] = g.reshape(1, 1, 1, size).repeat(channels, 1, 1, 1).to(device)
    return _WIN[key]


def _gfilter(x, win):
    c = x.shape[1]
    out = x
    for i, s in enumerate(x.shape[2:]):
        if s >= win.shape[-1]:
            out = F.conv2d(out, win.transpose(2 + i, -1), groups=c)
    return out


def ssim(x, y, data_range=1.0, win_size=11, win_sigma=1.5, K=(0.01, 0.03)):
    win = _window(win_size, win_sigma, x.shape[1], x.dtype, x.device)
    c1, c2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    mu1, mu2 = _gfilter(x, win), _gfilter(y, win)
    mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = _gfilter(x * x, win) - mu1_sq
    s2 = _gfilter(y * y, win) - mu2_sq
    s12 = _gfilter(x * y, win) - mu12
    cs_map = (2 * s12 + c2) / (s1 + s2 + c2)
    ssim_map = ((2 * mu12 + c1) / (mu1_sq + mu2_sq + c1)) * cs_map
    return torch.flatten(ssim_map, 2).mean(-1).mean()


def ssim_loss(x_hat, imgs):
    return 1 - ssim(x_hat, imgs, data_range=1)


def l1_loss(x_hat, imgs):
    return F.l1_loss(x_hat, imgs)
