"""VGG16 feature loss of MCM.forward_loss — counterpart of reference models/Compression/loss/vgg.py:9-115
(Vgg16 slices, feature_network, cal_features_loss) with common/image_utils.py:4-23 (de_normalize,
normalize_batch).

The reference rebuilds ``torchvision.models.vgg16(pretrained=True)`` on every call (a network download,
vgg.py:14, 99).  Here the frozen features[0:16] (relu1_2 / relu2_2 / relu3_3) are built ONCE from a LOCAL
VGG16 state_dict (torchvision key names ``features.N.weight``, or the reference Vgg16 module's
``sliceK.N.weight``), loaded with ``weights_only=True``; nothing is fetched.  The convolutions run on the
library's 3x3 conv kernels (NHWC, ReLU in the epilogue, tmae_conv3x3) and the loss backward on its conv
data-gradient kernel (tmae_conv_dgrad) plus the glue kernels of csrc/vgg.hip; the parameters stay frozen
(requires_grad=False in the reference), so only the gradient w.r.t. the prediction is formed.
"""
from __future__ import annotations

import warnings

import torch

from . import _lib, ops
from . import train_ops as T
from ._lib import ACT_RELU
from .ops import _stream

CONVS = (0, 2, 5, 7, 10, 12, 14)   # features[i] convs of slice1..slice3 (vgg.py:22-29)
POOL_AFTER = (2, 7)                # MaxPool2d follows features[3] (after conv 2) and features[8] (after conv 7)
CIN_PAD = 8                        # the RGB input padded to 8 channels (operand chunks of 8 bf16)


def _key(sd, i, what):
    for k in (f"features.{i}.{what}", f"{i}.{what}", f"slice1.{i}.{what}", f"slice2.{i}.{what}", f"slice3.{i}.{what}"):
        if k in sd:
            return sd[k]
    raise KeyError(f"VGG16 state_dict has no weight for features[{i}] ({what})")


def load_vgg16_state_dict(path):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd:
        sd = sd["state_dict"]
    return sd


class Vgg16Features:
    """frozen VGG16 features[0:16] on one device in one operand dtype"""

    def __init__(self, state_dict, device, dtype=torch.float32):
        self.device, self.dtype = torch.device(device), dtype
        self.w, self.wd, self.b, self.ch = [], [], [], []
        for i in CONVS:
            w = _key(state_dict, i, "weight").detach().float().to(self.device)
            b = _key(state_dict, i, "bias").detach().float().to(self.device).contiguous()
            cout, cin = w.shape[:2]
            if w.shape[2:] != (3, 3):
                raise ValueError(f"features[{i}] is not a 3x3 conv")
            cp = CIN_PAD if cin < CIN_PAD else cin
            wp = torch.zeros((cout, cp, 3, 3), device=self.device)
            wp[:, :cin] = w
            self.w.append(wp.permute(0, 2, 3, 1).reshape(cout, 9 * cp).to(dtype).contiguous())   # [Cout][3][3][Cin]
            self.wd.append(wp.permute(1, 2, 3, 0).reshape(cp, 9 * cout).to(dtype).contiguous())  # [Cin][3][3][Cout]
            self.b.append(b)
            self.ch.append((cp, cout))

    def _e(self, *shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.dtype, device=self.device)

    def forward(self, x, keep=False):
        """x: NCHW f32 image batch as the model sees it -> (relu2_2, relu3_3, saved) NHWC in the operand dtype"""
        x = x.float().contiguous()
        n, C, H, W = x.shape
        if H % 4 or W % 4:
            raise ValueError(f"VGG feature loss needs H, W divisible by 4 (got {H} x {W})")
        dt, code = self.dtype, ops.dtype_code(self.dtype)
        h = self._e(n * H * W, CIN_PAD)
        _lib.call("tmae_vgg_prep", x.data_ptr(), n, C, H, W, CIN_PAD, h.data_ptr(), code, _stream())
        saved = {"shape": (n, C, H, W), "acts": [], "args": []}
        cur, hh, ww = h, H, W
        feats = []
        for j, (cin, cout) in enumerate(self.ch):
            y = self._e(n * hh * ww, cout)
            # relu2_2 / relu3_3 feed the MSE: kept in f32 as well on the bf16 path (their difference is
            # small next to their magnitude)
            y32 = None
            if j in (3, 6):
                y32 = y if dt == torch.float32 else self._e(n * hh * ww, cout, dtype=torch.float32)
                feats.append(y32)
            ops.conv3x3(cur, cin, cin, n, hh, ww, self.w[j], self.b[j], y, cout, cout, dt, act=ACT_RELU,
                        y_f32=(dt == torch.float32), y32=None if y32 is y else y32, ld32=cout)
            saved["acts"].append((y, hh, ww))
            cur = y
            if CONVS[j] in POOL_AFTER:
                p = self._e(n * (hh // 2) * (ww // 2), cout)
                arg = torch.empty(p.numel(), dtype=torch.uint8, device=self.device) if keep else None
                _lib.call("tmae_maxpool2", cur.data_ptr(), n, hh, ww, cout, p.data_ptr(),
                          None if arg is None else arg.data_ptr(), code, _stream())
                saved["args"].append(arg)
                cur, hh, ww = p, hh // 2, ww // 2
        return feats[0], feats[1], (saved if keep else None)

    def backward(self, saved, g22, g33):
        """d loss / d x (NCHW f32) from the f32 gradients at relu2_2 and relu3_3 (NHWC)"""
        n, C, H, W = saved["shape"]
        dt, code = self.dtype, ops.dtype_code(self.dtype)
        if dt != torch.float32:  # the data gradients run in the operand dtype
            g22 = T.relayout(g22, torch.empty(g22.shape, dtype=dt, device=self.device), (g22.numel(),), (1,))
            g33 = T.relayout(g33, torch.empty(g33.shape, dtype=dt, device=self.device), (g33.numel(),), (1,))
        acts, args = saved["acts"], list(saved["args"])
        g = g33
        for j in reversed(range(len(self.ch))):
            cin, cout = self.ch[j]
            y, hh, ww = acts[j]
            _lib.call("tmae_relu_mask", g.data_ptr(), y.data_ptr(), y.numel(), code, _stream())
            dx = self._e(n * hh * ww, cin)
            T.conv_dgrad(g, self.wd[j], n, hh, ww, 1, cout, cin, dt, out=dx, out_f32=(dt == torch.float32))
            g = dx
            if j > 0 and CONVS[j - 1] in POOL_AFTER:   # the input of conv j is a pooled map
                yp, hp, wp = acts[j - 1]
                full = self._e(n * hp * wp, cin)
                add = g22 if j - 1 == 3 else None    # relu2_2 feeds the loss AND the next pool
                _lib.call("tmae_maxpool2_bwd", g.data_ptr(), args.pop().data_ptr(), n, hp, wp, cin, full.data_ptr(),
                          None if add is None else add.data_ptr(), code, _stream())
                g = full
        dx = torch.empty((n, C, H, W), dtype=torch.float32, device=self.device)
        _lib.call("tmae_vgg_prep_bwd", g.data_ptr(), n, C, H, W, CIN_PAD, dx.data_ptr(), code, _stream())
        return dx


_PART = {}


def _part(device):
    t = _PART.get(device)
    if t is None:
        t = _PART[device] = torch.empty(1024, dtype=torch.float64, device=device)
    return t


class FeatureLossFn(torch.autograd.Function):
    """cal_features_loss (vgg.py:86-115): MSE(relu2_2) + MSE(relu3_3) of VGG16(normalize(de_normalize(.)))"""

    @staticmethod
    def forward(ctx, preds, imgs, net):
        need = ctx.needs_input_grad[0]
        p22, p33, saved = net.forward(preds, keep=need)
        t22, t33, _ = net.forward(imgs, keep=False)
        code = ops.dtype_code(torch.float32)  # the features reach the MSE in f32
        out = torch.empty((), dtype=torch.float32, device=net.device)
        part = _part(net.device)
        _lib.call("tmae_mse", p22.data_ptr(), t22.data_ptr(), p22.numel(), part.data_ptr(), out.data_ptr(), 0, code,
                  _stream())
        _lib.call("tmae_mse", p33.data_ptr(), t33.data_ptr(), p33.numel(), part.data_ptr(), out.data_ptr(), 1, code,
                  _stream())
        if need:
            ctx.net, ctx.saved_state = net, saved
            ctx.feats = (p22, t22, p33, t33)
        return out

    @staticmethod
    def backward(ctx, g):
        net = ctx.net
        p22, t22, p33, t33 = ctx.feats
        code = ops.dtype_code(torch.float32)
        g = g.float().contiguous().reshape(1)
        g22, g33 = torch.empty_like(p22), torch.empty_like(p33)
        _lib.call("tmae_mse_bwd", p22.data_ptr(), t22.data_ptr(), p22.numel(), g.data_ptr(), g22.data_ptr(), code,
                  _stream())
        _lib.call("tmae_mse_bwd", p33.data_ptr(), t33.data_ptr(), p33.numel(), g.data_ptr(), g33.data_ptr(), code,
                  _stream())
        dx = net.backward(ctx.saved_state, g22, g33)
        ctx.saved_state = ctx.feats = None
        return dx, None, None


def cal_features_loss(preds, imgs, net):
    return FeatureLossFn.apply(preds, imgs, net)


_WARNED = [False]


def warn_missing_once():
    if not _WARNED[0]:
        _WARNED[0] = True
        warnings.warn("MCM.forward_loss: no local VGG16 weights (MCM.load_vgg16(path) or TMAE_VGG16_WEIGHTS); the "
                      "feature-loss term is 0, so RateDistortionLoss optimises lmbda*(0.25 ssim + 10 L1) + bpp only "
                      "(the reference downloads torchvision's pretrained VGG16, vgg.py:14)", stacklevel=3)
