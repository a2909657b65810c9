"""Distortion terms of MCM.forward_loss (reference MCM.py:690-712) on the HIP kernels of
csrc/distortion.hip: 1 - SSIM and L1 in one forward launch sequence, their backward in another.

SSIM follows pytorch_msssim (unpinned in the reference's requirements): 11-tap gaussian window,
sigma 1.5, valid separable filtering, K = (0.01, 0.03), data_range 1, mean over every channel map.
Images smaller than the window are filtered only along the dimensions that fit in pytorch_msssim;
the kernels need H, W >= 11 and raise otherwise.  The VGG term needs downloaded weights (vgg.py:14)
and is not computed.
"""
from __future__ import annotations

import torch

from . import _lib
from .ops import _stream

_PART = {}


def _part(device):
    t = _PART.get(device)
    if t is None:
        t = _PART[device] = torch.empty(2048, dtype=torch.float64, device=device)
    return t


class DistortionFn(torch.autograd.Function):
    """(x_hat, imgs) -> (1 - SSIM(x_hat, imgs), L1(x_hat, imgs)); gradient w.r.t. x_hat"""

    @staticmethod
    def forward(ctx, x_hat, imgs):
        x = x_hat.float().contiguous()
        y = imgs.float().contiguous()
        n, c, H, W = x.shape
        if H < 11 or W < 11:
            raise ValueError(f"SSIM needs images of at least 11x11 (got {H}x{W})")
        P = n * c
        need_grad = ctx.needs_input_grad[0]
        h = torch.empty(5 * P * H * (W - 10), dtype=torch.float32, device=x.device)
        d = torch.empty(3 * P * (H - 10) * (W - 10), dtype=torch.float32, device=x.device) if need_grad else None
        out = torch.empty(2, dtype=torch.float32, device=x.device)
        _lib.call("tmae_distortion_fwd", x.data_ptr(), y.data_ptr(), P, H, W, h.data_ptr(),
                  None if d is None else d.data_ptr(), _part(x.device).data_ptr(), out.data_ptr(), _stream())
        if need_grad:
            ctx.save_for_backward(x, y, d)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_ssim, g_l1):
        x, y, d = ctx.saved_tensors
        n, c, H, W = x.shape
        P = n * c
        dev = x.device
        gout = torch.stack([g_ssim.reshape(()) if g_ssim is not None else torch.zeros((), device=dev),
                            g_l1.reshape(()) if g_l1 is not None else torch.zeros((), device=dev)]).float().contiguous()
        v = torch.empty(3 * P * H * (W - 10), dtype=torch.float32, device=dev)
        gx = torch.empty_like(x)
        _lib.call("tmae_distortion_bwd", x.data_ptr(), y.data_ptr(), P, H, W, d.data_ptr(), v.data_ptr(),
                  gout.data_ptr(), gx.data_ptr(), _stream())
        return gx, None


def ssim_l1_loss(x_hat, imgs):
    """(1 - SSIM, L1) as 0-d device tensors (differentiable w.r.t. x_hat)"""
    return DistortionFn.apply(x_hat, imgs)


def ssim_loss(x_hat, imgs):
    return ssim_l1_loss(x_hat, imgs)[0]


def l1_loss(x_hat, imgs):
    return ssim_l1_loss(x_hat, imgs)[1]
