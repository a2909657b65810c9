"""MCM — drop-in for reference models/Compression/MCM.py:25 (``class MCM(CompressionModel)``).

Same constructor arguments and defaults (MCM.py:34-52), same submodule names, so
``state_dict()`` keys, ``named_parameters()`` (``*.quantiles`` split, model_utils.py:67-90) and
``load_state_dict`` behave as in the reference; same call surface (``forward(imgs, total_scores)``
-> ``{"loss", "likelihoods", "x_hat"}``, ``aux_loss()``, ``from_state_dict``, ``patchify`` /
``unpatchify``).

Underneath, ``forward`` never calls a PyTorch compute op on the hot path: it enqueues the gfx950
kernels of libtmae.so on the current stream through a persistent workspace (``_Executor``), with
the LIC feature maps kept NHWC end to end.  ``compute_dtype`` selects the MFMA
operand type: torch.float32 (exact f32 MFMA; the parity path, default) or torch.bfloat16
(throughput path; f32 accumulate, f32 residual stream / entropy models / likelihoods).
"""
from __future__ import annotations

import os

from functools import partial

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .entropy import CompressionModel, EntropyBottleneck, GaussianConditional
from .layers import Block, BlockScratch, BlockWeights, PatchEmbed, conv3x3, run_block, subpel_conv3x3
from .pos_embed import get_2d_sincos_pos_embed


class MCM(CompressionModel):
    """Masked-compression model: MAE-ViT encoder -> hyperprior LIC with channel-conditional slices ->
    MAE-ViT decoder (reference MCM.py:25-968)."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, encoder_embed_dim=768, encoder_depth=12,
                 encoder_num_heads=12, decoder_embed_dim=512, decoder_depth=8, decoder_num_heads=16, mlp_ratio=4.0,
                 norm_layer=partial(nn.LayerNorm, eps=1e-6), norm_pix_loss=False, latent_depth=384,
                 hyperprior_depth=192, num_slices=12, num_keep_patches=144):
        super().__init__()
        self.frozen_stages = -1
        self.encoder_embed_dim = E = encoder_embed_dim
        self.encoder_depth = encoder_depth
        self.encoder_num_heads = encoder_num_heads
        self.decoder_embed_dim = Dd = decoder_embed_dim
        self.decoder_depth = decoder_depth
        self.decoder_num_heads = decoder_num_heads
        self.latent_depth = M = latent_depth
        self.hyperprior_depth = N = hyperprior_depth
        self.num_slices = S = num_slices
        self.num_keep_patches = num_keep_patches

        # entropy models (MCM.py:71-73)
        self.entropy_bottleneck = EntropyBottleneck(N)
        self.gaussian_conditional = GaussianConditional(None)
        self.max_support_slices = S // 2

        # g_a / g_s: 1x1 convs E -> .. -> M and back (MCM.py:77-112)
        ga = [E, int(Dd + (E - Dd) * 3 / 4), int(Dd + (E - Dd) * 2 / 4), Dd, M]
        self.g_a = nn.Sequential(*_interleave([nn.Conv2d(ga[j], ga[j + 1], 1, 1, 0) for j in range(4)]))
        gs = ga[::-1]
        self.g_s = nn.Sequential(*_interleave([nn.ConvTranspose2d(gs[j], gs[j + 1], 1, 1, 0) for j in range(4)]))

        # h_a / h_s (MCM.py:115-162)
        ha = [M, M, int(N + (M - N) * 3 / 4), int(N + (M - N) * 2 / 4), int(N + (M - N) / 4), N]
        self.h_a = nn.Sequential(*_interleave([conv3x3(ha[j], ha[j + 1], stride=(2 if j in (2, 4) else 1))
                                               for j in range(5)]))
        hs = [N, int(N + (M - N) / 4), int(N + (M - N) * 2 / 4), int(N + (M - N) * 3 / 4), M, M]

        def h_s():
            return nn.Sequential(*_interleave([
                conv3x3(hs[0], hs[1]), subpel_conv3x3(hs[1], hs[2], r=2), conv3x3(hs[2], hs[3]),
                subpel_conv3x3(hs[3], hs[4], r=2), conv3x3(hs[4], hs[5])]))

        self.h_s_mean = h_s()
        self.h_s_scale = h_s()

        # channel-conditional slice transforms (MCM.py:165-293)
        sw = M // S
        mid = [int(sw * (S // 2 + 1)), int(sw * (S // 2 * 3 / 4 + 1)), int(sw * (S // 2 * 2 / 4 + 1)),
               int(sw * (S // 2 * 1 / 4 + 1)), sw]

        def stack(cin):
            ch = [cin] + mid
            return nn.Sequential(*_interleave([nn.Conv2d(ch[j], ch[j + 1], 3, 1, 1) for j in range(5)]))

        self.cc_transform_mean = nn.ModuleList([stack(int(M + sw * min(i, S // 2))) for i in range(S)])
        self.cc_transform_scale = nn.ModuleList([stack(int(M + sw * min(i, S // 2))) for i in range(S)])
        self.lrp_transform = nn.ModuleList([stack(int(M + sw * min(i + 1, S // 2 + 1))) for i in range(S)])

        # MAE encoder / decoder (MCM.py:300-354)
        self.encoder_embed = PatchEmbed(img_size, patch_size, in_chans, E)
        num_patches = self.encoder_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, E))
        self.encoder_pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, E), requires_grad=False)
        self.encoder_blocks = nn.ModuleList([Block(dim=E, num_heads=encoder_num_heads, mlp_ratio=mlp_ratio,
                                                   qkv_bias=True, norm_layer=norm_layer)
                                             for _ in range(encoder_depth)])
        self.encoder_norm = norm_layer(E)
        self.decoder_embed = nn.Linear(E, Dd, bias=True)
        self.mask_token = nn.Parameter(torch.zeros(1, 1, Dd))
        self.decoder_pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, Dd), requires_grad=False)
        self.decoder_blocks = nn.ModuleList([Block(dim=Dd, num_heads=decoder_num_heads, mlp_ratio=mlp_ratio,
                                                   qkv_bias=True, norm_layer=norm_layer)
                                             for _ in range(decoder_depth)])
        self.decoder_norm = norm_layer(Dd)
        self.decoder_pred = nn.Linear(Dd, patch_size ** 2 * in_chans, bias=True)
        self.norm_pix_loss = norm_pix_loss
        self.initialize_weights()

        # MI355X execution settings (not part of the reference surface)
        self.compute_dtype = torch.float32
        self.sum_lanes = 8          # torch CPU float-sum vector width the reference ran with
        self.distortion = "ssim+l1"  # forward_loss terms; "none" skips them (encode/decode/rate only)
        self._exec = None

    # ---------------------------------------------------------------------------------- init
    def initialize_weights(self):
        """MCM.initialize_weights / _init_weights (MCM.py:454-495)."""
        g = int(self.encoder_embed.num_patches ** 0.5)
        self.encoder_pos_embed.data.copy_(
            torch.from_numpy(get_2d_sincos_pos_embed(self.encoder_pos_embed.shape[-1], g, True)).float().unsqueeze(0))
        self.decoder_pos_embed.data.copy_(
            torch.from_numpy(get_2d_sincos_pos_embed(self.decoder_pos_embed.shape[-1], g, True)).float().unsqueeze(0))
        w = self.encoder_embed.proj.weight.data
        torch.nn.init.xavier_uniform_(w.view([w.shape[0], -1]))
        torch.nn.init.normal_(self.cls_token, std=0.02)
        torch.nn.init.normal_(self.mask_token, std=0.02)
        self.apply(self._init_weights)

    @staticmethod
    def _init_weights(m):
        if isinstance(m, nn.Linear):
            torch.nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def load_state_dict(self, state_dict, strict=True):
        # the reference override drops `strict` (MCM.py:445-446); keep the compressai buffer resizing
        r = super().load_state_dict(state_dict, strict=strict)
        self._exec = None
        self._train_exec = None
        return r

    @classmethod
    def from_state_dict(cls, num_keep_patches, state_dict):
        net = cls(num_keep_patches=num_keep_patches)
        net.load_state_dict(state_dict)
        return net

    # ---------------------------------------------------------------------------------- layout helpers
    def patchify(self, imgs):
        p = self.encoder_embed.patch_size[0]
        assert imgs.shape[2] == imgs.shape[3] and imgs.shape[2] % p == 0
        h = w = imgs.shape[2] // p
        x = imgs.reshape(imgs.shape[0], 3, h, p, w, p)
        return torch.einsum("nchpwq->nhwpqc", x).reshape(imgs.shape[0], h * w, p ** 2 * 3)

    def unpatchify(self, x):
        p = self.encoder_embed.patch_size[0]
        h = w = int(x.shape[1] ** 0.5)
        assert h * w == x.shape[1]
        x = torch.einsum("nhwpqc->nchpwq", x.reshape(x.shape[0], h, w, p, p, 3))
        return x.reshape(x.shape[0], 3, h * p, w * p)

    # ---------------------------------------------------------------------------------- masking
    def get_ids_shuffle(self, total_scores):
        """MCM.get_ids_shuffle (MCM.py:364-423) — one GPU launch for the whole batch."""
        if self.num_keep_patches > total_scores.shape[1]:
            raise ValueError("Number of patches should not be greater than the length of scores")
        return ops.ids_shuffle(total_scores, self.num_keep_patches, self.sum_lanes)[0]

    def random_masking(self, x, total_scores):
        """MCM.random_masking (MCM.py:548-588): (x_remain, ids_restore)."""
        shuf, rest = ops.ids_shuffle(total_scores, self.num_keep_patches, self.sum_lanes)
        D = x.shape[-1]
        x_remain = torch.gather(x, 1, shuf[:, : self.num_keep_patches].unsqueeze(-1).repeat(1, 1, D))
        return x_remain, rest

    # ---------------------------------------------------------------------------------- forward
    def _executor(self, batch, device):
        dt = self.compute_dtype
        if torch.is_autocast_enabled() and dt == torch.float32:
            dt = torch.bfloat16  # val_one_epoch runs under autocast (utils/engine.py:189)
        ex = self._exec
        if ex is None or ex.batch != batch or ex.dtype != dt or ex.device != device:
            ex = self._exec = _Executor(self, batch, dt, device)
        ex.refresh_weights()
        return ex

    def forward(self, imgs, total_scores, noise=None):
        """MCM.forward (MCM.py:714-803).  `noise=(z_noise, y_noise)` (NCHW, U(-1/2, 1/2)) replaces the
        training-mode quantisation noise — used by parity tests; otherwise drawn on the device."""
        if not imgs.is_cuda:
            raise ValueError("MCM.forward runs on the MI355X kernels: move the model and inputs to the GPU")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return self._forward_train(imgs, total_scores, noise)
        with torch.no_grad():
            ex = self._executor(imgs.shape[0], imgs.device)
            out = ex.run(imgs, total_scores, self.training, noise)
            x_hat = out["x_hat"]
            loss = self.forward_loss(imgs, x_hat) if self.distortion != "none" else (ex.zero_loss,) * 3
        return {"loss": loss, "likelihoods": {"y": out["y"], "z": out["z"]}, "x_hat": x_hat}

    def _forward_train(self, imgs, total_scores, noise):
        """MCM.forward under autograd (utils/engine.py:75): one autograd node whose forward keeps the
        activations and whose backward is the HIP reverse pass (mcm_train.py)."""
        from .mcm_train import TrainExec, _MCMTrainFn

        dt = self.compute_dtype
        if torch.is_autocast_enabled() and dt == torch.float32:
            dt = torch.bfloat16
        B = imgs.shape[0]
        ex = getattr(self, "_train_exec", None)
        if ex is None or ex.batch != B or ex.dtype != dt or ex.device != imgs.device:
            ex = self._train_exec = TrainExec(self, B, dt, imgs.device)
        x_hat, ylik, zlik = _MCMTrainFn.apply(ex, noise, imgs, total_scores, *self.parameters())
        loss = self.forward_loss(imgs, x_hat) if self.distortion != "none" else (
            torch.zeros((), device=imgs.device),) * 3
        return {"loss": loss, "likelihoods": {"y": ylik, "z": zlik}, "x_hat": x_hat}

    def forward_loss(self, imgs, x_hat):
        """MCM.forward_loss (MCM.py:690-712): (1 - SSIM, L1, VGG16 feature loss).  The reference downloads
        torchvision's pretrained VGG16 on every call (vgg.py:14, 99); here the feature loss runs once local
        weights are given (load_vgg16, or the TMAE_VGG16_WEIGHTS file) and is 0 (with a one-time warning in
        training) without them."""
        from . import vgg
        from .distortion import ssim_l1_loss

        s, l1 = ssim_l1_loss(x_hat, imgs)
        net = self._vgg_net(imgs.device)
        if net is None:
            if self.training:
                vgg.warn_missing_once()
            return s, l1, torch.zeros((), device=imgs.device)
        return s, l1, vgg.cal_features_loss(x_hat, imgs, net)

    def load_vgg16(self, weights):
        """local VGG16 weights for the feature loss: a torchvision vgg16 state_dict (or the reference Vgg16
        module's) or a path to one (loaded with weights_only=True).  Not part of MCM's state_dict, as in the
        reference, where the network is frozen and rebuilt inside the loss."""
        from .vgg import load_vgg16_state_dict

        sd = load_vgg16_state_dict(weights) if isinstance(weights, (str, os.PathLike)) else weights
        self.__dict__["_vgg_sd"] = {k: v.detach().cpu() for k, v in sd.items() if torch.is_tensor(v)}
        self.__dict__["_vgg"] = None

    def _vgg_net(self, device):
        from .vgg import Vgg16Features

        if self.__dict__.get("_vgg_sd") is None:
            path = os.environ.get("TMAE_VGG16_WEIGHTS")
            if not path:
                return None
            self.load_vgg16(path)
        dt = self.compute_dtype
        if torch.is_autocast_enabled() and dt == torch.float32:
            dt = torch.bfloat16
        net = self.__dict__.get("_vgg")
        if net is None or net.device != torch.device(device) or net.dtype != dt:
            net = Vgg16Features(self.__dict__["_vgg_sd"], device, dt)
            self.__dict__["_vgg"] = net
        return net

    def aux_loss(self):
        return self.entropy_bottleneck.loss()

    def compress(self, imgs, total_scores):
        """MCM.compress (MCM.py:805-894) -> {"string": [[y_string], z_strings], "shape", "ids_restore"}.
        Needs the CDF tables: call update(force=True) first (testing.py:223), as with compressai."""
        if not imgs.is_cuda:
            raise ValueError("MCM.compress runs on the MI355X kernels: move the model and inputs to the GPU")
        self.entropy_bottleneck._check_cdf()
        self.gaussian_conditional._check_cdf()
        with torch.no_grad():
            ex = self._executor(imgs.shape[0], imgs.device)
            return ex.compress(imgs, total_scores)

    def decompress(self, strings, shape, ids_restore=None):
        """MCM.decompress (MCM.py:896-968) -> {"x_hat"}.  Batch = number of z strings; the reference's
        reshape(1, ...) at MCM.py:944 limits it to one image, this handles any batch the y string holds."""
        assert isinstance(strings, list) and len(strings) == 2
        if ids_restore is None:
            raise ValueError("MCM.decompress needs ids_restore (the decoder unshuffles by it, MCM.py:667-669)")
        self.entropy_bottleneck._check_cdf()
        self.gaussian_conditional._check_cdf()
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise ValueError("MCM.decompress runs on the MI355X kernels: move the model to the GPU")
        with torch.no_grad():
            ex = self._executor(len(strings[1]), dev)
            return {"x_hat": ex.decompress(strings, shape, ids_restore)}


def _interleave(layers):
    out = []
    for j, l in enumerate(layers):
        out.append(l)
        if j < len(layers) - 1:
            out.append(nn.GELU())
    return out


# ====================================================================================== executor
class _Executor:
    """Prepared weights + persistent workspaces for one (batch, dtype, device); `run` enqueues the
    whole forward on the current stream (graph-capturable: no host sync, no allocation-dependent
    control flow).

    LIC slice loop restructure (exact up to f32 summation order):
      * the first conv of every cc_transform_mean/scale and lrp_transform stack sees
        cat(latent_{means,scales}, y_hat slices): its latent-channel part is the same input for all 12
        slices, so it is computed for all slices up front as two big convs (N = 3 * 12 * 224) into the
        partial-sum buffer P; each slice's first conv then only contracts the y_hat channels and adds
        its P block in the epilogue;
      * the mean and scale stacks of a slice run as one batched launch per layer;
      * slices 6..11 all condition on y_hat slices 0..5 (max_support_slices = 6, MCM.py:73, 756-758),
        so their mean/scale stacks, Gaussian likelihoods and lrp stacks run batched (12 / 6 problems).
    """

    # reference paths the tests compare the fused LIC launches against (bitwise / bounded): False selects the
    # per-layer conv launches (the f32 parity path's structure) or the unchained serial slices
    USE_LIC_STACK = True
    USE_LIC_CHAIN = True
    USE_LIC_LATENT = True  # False: the latent partial sums on the halo conv (conv_halo.h)

    def __init__(self, m: MCM, batch, dtype, device):
        self.m, self.batch, self.dtype, self.device = m, batch, dtype, device
        self._sig = None
        B = batch
        E, Dd, M, N, S = m.encoder_embed_dim, m.decoder_embed_dim, m.latent_depth, m.hyperprior_depth, m.num_slices
        K = m.num_keep_patches
        P = m.encoder_embed.patch_size[0]
        self.img = m.encoder_embed.img_size[0]
        self.P, self.L = P, m.encoder_embed.num_patches
        self.g = g = int(round(K ** 0.5))
        if g * g != K:
            raise ValueError(f"num_keep_patches={K} must be a perfect square (MCM.py:729-732 views it as sqrt x sqrt)")
        self.hz = ((g + 1) // 2 + 1) // 2  # two stride-2 convs
        if self.hz * 4 != g:
            raise ValueError(f"sqrt(num_keep_patches)={g} must be a multiple of 4 so h_s returns to the y grid")
        self.sw = M // S
        self.maxsup = S // 2
        self.nb = S - self.maxsup  # slices sharing the full support (batched)
        f32, dt = torch.float32, dtype
        dev = device

        def z(*shape, dtype=f32):
            return torch.empty(shape, dtype=dtype, device=dev)

        Te, Td = K + 1, self.L + 1
        Mp = B * g * g
        self.Mp = Mp
        hid_e = m.encoder_blocks[0].mlp.fc1.out_features if m.encoder_depth else 4 * E
        hid_d = m.decoder_blocks[0].mlp.fc1.out_features if m.decoder_depth else 4 * Dd
        self.tok = z(B * Te, E)
        self.enc_s = BlockScratch(B * Te, E, hid_e, dt, dev)
        self.enc_out = z(B * K, E, dtype=dt)
        ga = [l.out_channels for l in m.g_a if isinstance(l, nn.Conv2d)]
        self.ga_buf = [z(B * K, c, dtype=dt) for c in ga[:-1]]
        self.Y32 = z(Mp, M)
        self.YT = self.Y32 if dt == f32 else z(Mp, M, dtype=dt)
        ha = [l.out_channels for l in m.h_a if isinstance(l, nn.Conv2d)]
        res = [g, g, (g + 1) // 2, (g + 1) // 2, self.hz]
        self.ha_buf = [z(B * r * r, c, dtype=dt) for c, r in zip(ha[:-1], res[:-1])]
        self.Z = z(B * self.hz * self.hz, N)
        self.ZLIK = z(B, N, self.hz, self.hz)
        self.ZHAT = z(B * self.hz * self.hz, N, dtype=dt)
        self.eb_table = z(N, 59)
        self.zero_loss = torch.zeros((), device=device)  # the loss terms of distortion="none" (never written)
        hs_out = [m.h_s_mean[0].out_channels, m.h_s_mean[2][0].out_channels // 4, m.h_s_mean[4].out_channels,
                  m.h_s_mean[6][0].out_channels // 4]
        hs_res = [self.hz, 2 * self.hz, 2 * self.hz, g]
        # h_s_scale / h_s_mean run as one 2-problem launch per layer: [scale, mean] slabs
        self.hs_buf = [z(2, B * r * r, c, dtype=dt) for c, r in zip(hs_out, hs_res)]
        self.LSM = z(2, Mp, M, dtype=dt)
        self.LS, self.LM = self.LSM[0], self.LSM[1]
        self.mid = [l.out_channels for l in m.cc_transform_mean[0] if isinstance(l, nn.Conv2d)]
        c0 = self.mid[0]
        self.PW = 3 * S * c0  # partial sums: [mean (S*c0) | lrp (S*c0) | scale (S*c0)]
        self.Pbuf = z(Mp, self.PW)
        # side stream for the partial sums under the serial slice steps (_slices)
        self.overlap = torch.device(dev).type == "cuda"
        self.side_stream = torch.cuda.Stream(device=dev) if self.overlap else None
        self.SUPY = z(Mp, M, dtype=dt)    # y_hat slices (post-LRP for i < maxsup; pre-LRP for the batched ones)
        self.YPRE = z(Mp, M)              # f32 pre-LRP y_hat = round(y - mu) + mu
        self.YH = z(Mp, M, dtype=dt)      # final y_hat (g_s input)
        nb = self.nb
        self.CM = [z(2, nb, Mp, c, dtype=dt) for c in self.mid[:-1]]
        self.MUSIG = z(2, nb, Mp, self.sw)
        # chained serial slices (mean stack + lrp stack in one launch): every serial slice's mu / sigma kept
        # for the one deferred likelihood launch after the slice loop
        self.MS_SER = z(2, S, Mp, self.sw)
        self.CL = [z(nb, Mp, c, dtype=dt) for c in self.mid[:-1]]
        self.YLIK = z(B, M, g, g)
        gs = [l.out_channels for l in m.g_s if isinstance(l, nn.ConvTranspose2d)]
        self.gs_buf = [z(B * K, c, dtype=dt) for c in gs]
        self.dec = z(B * Td, Dd)
        self.dec_s = BlockScratch(B * Td, Dd, hid_d, dt, dev)
        self.dn = z(B * self.L, Dd, dtype=dt)

    # ------------------------------------------------------------------ weights
    def refresh_weights(self):
        sig = tuple((p.data_ptr(), p._version) for p in self.m.parameters())
        if sig == self._sig:
            return
        self._sig = sig
        m, dt = self.m, self.dtype
        M, S, sw, ms = m.latent_depth, m.num_slices, self.sw, self.maxsup

        def cast(t):
            t = t.detach()
            return (t if dt == torch.float32 else t.to(dt)).contiguous()

        def cw(w, lo=None, hi=None):  # conv weight [Cout][Cin][3][3] -> [Cout][3][3][Cin slice]
            w = w.detach()
            if lo is not None:
                w = w[:, lo:hi]
            return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)

        self.w_pe = cast(m.encoder_embed.proj.weight.view(m.encoder_embed.proj.weight.shape[0], -1))
        self.enc_w = [BlockWeights.from_block(b, dt) for b in m.encoder_blocks]
        self.dec_w = [BlockWeights.from_block(b, dt) for b in m.decoder_blocks]
        self.ga_w = [(cast(l.weight.view(l.weight.shape[0], -1)), l.bias.detach())
                     for l in m.g_a if isinstance(l, nn.Conv2d)]
        self.gs_w = [(cast(l.weight.view(l.weight.shape[0], -1).t()), l.bias.detach())
                     for l in m.g_s if isinstance(l, nn.ConvTranspose2d)]
        self.ha_w = [(cast(cw(l.weight)), l.bias.detach(), l.stride[0]) for l in m.h_a if isinstance(l, nn.Conv2d)]

        def hs_convs(seq):  # (conv, followed by PixelShuffle) of h_s_mean / h_s_scale
            out = []
            for l in seq:
                if isinstance(l, nn.Conv2d):
                    out.append((l, False))
                elif isinstance(l, nn.Sequential):
                    out.append((l[0], True))
            return out

        # [scale, mean] weights / biases of each layer stacked for the 2-problem launch
        self.hs2_w = [(cast(torch.stack([cw(s.weight), cw(mn.weight)])),
                       torch.stack([s.bias, mn.bias]).detach().contiguous(), ps)
                      for (s, ps), (mn, _) in zip(hs_convs(m.h_s_scale), hs_convs(m.h_s_mean))]

        def convs(seq):
            return [l for l in seq if isinstance(l, nn.Conv2d)]

        mean = [convs(s) for s in m.cc_transform_mean]
        scale = [convs(s) for s in m.cc_transform_scale]
        lrp = [convs(s) for s in m.lrp_transform]
        # latent-channel parts of every first conv: [mean | lrp] from latent_means, scale from latent_scales
        self.w_pre_ml = cast(torch.cat([cw(mean[i][0].weight, 0, M) for i in range(S)]
                                       + [cw(lrp[i][0].weight, 0, M) for i in range(S)]))
        self.w_pre_s = cast(torch.cat([cw(scale[i][0].weight, 0, M) for i in range(S)]))
        # the same latent parts in fragment order, one block per stack [mean | lrp | scale] x slices (tmae_lic_latent)
        c0 = self.mid[0]
        self.w_lat = None
        if dt == torch.bfloat16 and self.USE_LIC_LATENT and ops.lic_latent_fits(self.g, M) and c0 % 32 == 0:
            self.w_lat = torch.stack([ops.pack_lic_stack_weight(t[i][0].weight[:, :M])
                                      for t in (mean, lrp, scale) for i in range(S)]).contiguous()
        # per-slice y_hat-channel parts + the remaining layers, packed for batched launches
        self.ms_first, self.ms_layers, self.lrp_first, self.lrp_layers = [], [], [], []
        for i in range(ms):
            ny = sw * i
            self.ms_first.append((cast(torch.stack([cw(mean[i][0].weight, M, M + ny), cw(scale[i][0].weight, M, M + ny)])),
                                  torch.stack([mean[i][0].bias, scale[i][0].bias]).detach().contiguous()))
            self.ms_layers.append([(cast(torch.stack([cw(mean[i][j].weight), cw(scale[i][j].weight)])),
                                    torch.stack([mean[i][j].bias, scale[i][j].bias]).detach().contiguous())
                                   for j in range(1, 5)])
            self.lrp_first.append((cast(cw(lrp[i][0].weight, M, M + ny + sw)), lrp[i][0].bias.detach()))
            self.lrp_layers.append([(cast(cw(lrp[i][j].weight)), lrp[i][j].bias.detach()) for j in range(1, 5)])
        bs = range(ms, S)
        ny = sw * ms
        self.b_ms_first = (cast(torch.stack([torch.stack([cw(t[i][0].weight, M, M + ny) for i in bs])
                                             for t in (mean, scale)])),
                           torch.stack([torch.stack([t[i][0].bias for i in bs]) for t in (mean, scale)]).detach()
                           .contiguous())
        self.b_ms_layers = [(cast(torch.stack([torch.stack([cw(t[i][j].weight) for i in bs]) for t in (mean, scale)])),
                             torch.stack([torch.stack([t[i][j].bias for i in bs]) for t in (mean, scale)]).detach()
                             .contiguous()) for j in range(1, 5)]
        self.b_lrp_first = (cast(torch.stack([cw(lrp[i][0].weight, M, M + ny + sw) for i in bs])),
                            torch.stack([lrp[i][0].bias for i in bs]).detach().contiguous())
        self.b_lrp_layers = [(cast(torch.stack([cw(lrp[i][j].weight) for i in bs])),
                              torch.stack([lrp[i][j].bias for i in bs]).detach().contiguous()) for j in range(1, 5)]
        # fused slice-transform stacks (lic_stack.hip): every layer packed in MFMA fragment order, problems
        # stacked like the per-layer launches above; bf16 only, shapes that fit one workgroup's LDS
        self.lstk = None
        if (dt == torch.bfloat16 and self.USE_LIC_STACK and sw % 8 == 0
                and ops.lic_stack_fits(self.g, sw * (ms + 1), self.mid)):
            pk = ops.pack_lic_stack_weight

            def packs(convs, lo=None, hi=None):  # [layer] -> packed weights of one stack
                return [pk(c.weight[:, lo:hi] if j == 0 else c.weight) for j, c in enumerate(convs)]

            def stk(ts):  # stack problems' packed weights per layer
                return [torch.stack(list(layer)).contiguous() for layer in zip(*ts)]

            L = {"ms": [], "lrp": []}
            for i in range(ms):
                ny = sw * i
                L["ms"].append(stk([packs(mean[i], M, M + ny), packs(scale[i], M, M + ny)]))
                L["lrp"].append(packs(lrp[i], M, M + ny + sw))
            if S > ms:
                ny = sw * ms
                L["b_ms"] = [torch.stack([a_, b_]).contiguous() for a_, b_ in
                             zip(stk([packs(mean[i], M, M + ny) for i in bs]), stk([packs(scale[i], M, M + ny) for i in bs]))]
                L["b_lrp"] = stk([packs(lrp[i], M, M + ny + sw) for i in bs])
            self.lstk = L
        self.w_de = cast(m.decoder_embed.weight)
        # decoder_pred rows in channel-planar order: the unpatchify epilogue stores whole pixel runs
        pp = m.encoder_embed.patch_size[0]
        perm = ops.pred_channel_planar_perm(pp, m.encoder_embed.proj.in_channels)
        pred_cp = pp % 8 == 0
        self.pred_cp = pred_cp
        self.w_dp = cast(m.decoder_pred.weight[perm.to(m.decoder_pred.weight.device)] if pred_cp
                         else m.decoder_pred.weight)
        self.b_dp = (m.decoder_pred.bias[perm.to(m.decoder_pred.bias.device)] if pred_cp
                     else m.decoder_pred.bias).detach().contiguous()

    # ------------------------------------------------------------------ forward
    def _check_imgs(self, imgs):
        imgs = imgs.float().contiguous()
        if imgs.shape[1:] != (self.m.encoder_embed.proj.in_channels, self.img, self.img):
            raise ValueError(f"Input image size {tuple(imgs.shape[2:])} doesn't match model ({self.img})")
        return imgs

    def run(self, imgs, scores, training, noise):
        m, B = self.m, self.batch
        M, N, g, hz = m.latent_depth, m.hyperprior_depth, self.g, self.hz
        imgs = self._check_imgs(imgs)
        if training:
            if noise is not None:
                z_noise, y_noise = (t.float().contiguous() for t in noise)
            else:
                z_noise = torch.empty((B, N, hz, hz), device=self.device).uniform_(-0.5, 0.5)
                y_noise = torch.empty((B, M, g, g), device=self.device).uniform_(-0.5, 0.5)
        else:
            z_noise = y_noise = None

        # the likelihoods are returned to the caller: fresh tensors per forward (no copy of the executor's)
        self.ZLIK = torch.empty_like(self.ZLIK)
        self.YLIK = torch.empty_like(self.YLIK)
        shuf, rest = self._front(imgs, scores)

        # ---- entropy bottleneck + z_hat (MCM.py:741-744)
        ops.eb_likelihood(m.entropy_bottleneck, self.Z, B, N, hz * hz, noise=z_noise, lik=self.ZLIK, zhat=self.ZHAT,
                          table=self.eb_table)

        # ---- h_s (MCM.py:747-748)
        self._h_s()

        # ---- slice loop (MCM.py:751-787)
        self._slices(self._gc_forward(y_noise), chain_ok=True)

        x_hat = self._back(shuf, imgs.shape[1])
        return {"x_hat": x_hat, "y": self.YLIK, "z": self.ZLIK, "ids_restore": rest,
                "ids_shuffle": shuf}

    # ------------------------------------------------------------------ compress / decompress
    def compress(self, imgs, scores):
        """MCM.compress (MCM.py:805-894): the eval forward's analysis path with symbol/index outputs, then
        the host rANS coder: one z string per image, ONE y string for the whole batch (slice-major)."""
        from .coder import BufferedRansEncoder

        m, B = self.m, self.batch
        N, S, hz, sw, HW = m.hyperprior_depth, m.num_slices, self.hz, self.sw, self.g * self.g
        eb, gc = m.entropy_bottleneck, m.gaussian_conditional
        imgs = self._check_imgs(imgs)
        shuf, rest = self._front(imgs, scores)
        # z: symbols round(z - median); z_hat = symbols + median (= EB.decompress of its own strings)
        ops.eb_likelihood(eb, self.Z, B, N, hz * hz, lik=self.ZLIK, zhat=self.ZHAT, table=self.eb_table)
        zsym = ops.eb_symbols(eb, self.Z, B, N, hz * hz, table=self.eb_table)
        self._h_s()
        sym = torch.empty(S * B * sw * HW, dtype=torch.int32, device=self.device)
        idx = torch.empty_like(sym)
        self._slices(self._gc_compress(sym, idx))
        zsym_h, sym_h, idx_h = zsym.cpu().numpy(), sym.cpu().numpy(), idx.cpu().numpy()
        self.last_streams = {"z_symbols": zsym_h, "y_symbols": sym_h, "y_indexes": idx_h}  # rate diagnostics
        zidx = eb._channel_indexes(hz * hz)
        z_strings = [eb._code(zsym_h[b].reshape(-1), zidx) for b in range(B)]
        enc = BufferedRansEncoder()
        enc.encode_with_indexes(sym_h, idx_h, *gc.host_tables())
        return {"string": [[enc.flush()], z_strings], "shape": torch.Size([hz, hz]), "ids_restore": rest}

    def decompress(self, strings, shape, ids_restore):
        """MCM.decompress (MCM.py:896-968): z strings -> z_hat -> h_s -> slice loop decoding each slice's
        symbols from the y string with indexes built on the device -> g_s -> decoder."""
        from .coder import RansDecoder

        m, B = self.m, self.batch
        N, hz = m.hyperprior_depth, self.hz
        eb = m.entropy_bottleneck
        if tuple(int(v) for v in shape) != (hz, hz):
            raise ValueError(f"shape {tuple(shape)} does not match this model's z grid ({hz}, {hz})")
        zidx = eb._channel_indexes(hz * hz)
        zsym = np.stack([eb._decode(s, zidx) for s in strings[1]]).astype(np.int32)
        ops.eb_dequantize(eb, torch.from_numpy(zsym).to(self.device), B, N, hz * hz, self.ZHAT, table=self.eb_table)
        self._h_s()
        decoder = RansDecoder()
        decoder.set_stream(strings[0][0])
        self._slices(self._gc_decompress(decoder))
        shuf = ops.invert_permutation(ids_restore.to(self.device))
        return self._back(shuf, m.encoder_embed.proj.in_channels)

    def _front(self, imgs, scores):
        """encoder + g_a + h_a (MCM.py:590-634, 729-739): tokens -> Y32/YT -> Z; returns (ids_shuffle, ids_restore)"""
        m, dt, B = self.m, self.dtype, self.batch
        E, M, K, P, g = m.encoder_embed_dim, m.latent_depth, m.num_keep_patches, self.P, self.g
        Te = K + 1
        # ---- encoder (MCM.py:590-634): ids on device, embed only the kept patches
        shuf, rest = ops.ids_shuffle(scores, K, m.sum_lanes)
        pos_e = m.encoder_pos_embed.detach()
        ops.patch_embed(imgs, shuf, self.w_pe, m.encoder_embed.proj.bias.detach(), pos_e, self.tok, K, P, dt)
        ops.cls_rows(self.tok, m.cls_token.detach(), pos_e, B, Te, E)
        for w in self.enc_w:
            run_block(self.tok, w, B, Te, dt, self.enc_s)
        ops.layernorm(self.tok, m.encoder_norm.weight, m.encoder_norm.bias, m.encoder_norm.eps, dt, rows=B * K,
                      row_group=K, group_stride=Te, row_offset=1, out=self.enc_out)

        # ---- g_a: 1x1 convs on the token matrix (tokens in ids_keep order = the g x g grid, MCM.py:729-735)
        x = self.enc_out
        for j, (w, b) in enumerate(self.ga_w):
            last = j == len(self.ga_w) - 1
            if last:
                ops.linear(x, w, b, dt, out=self.YT, out32=None if self.YT is self.Y32 else self.Y32)
            else:
                ops.linear(x, w, b, dt, act=ops.ACT_GELU, out=self.ga_buf[j])
                x = self.ga_buf[j]

        # ---- h_a (MCM.py:739)
        H = g
        x, cin = self.YT, M
        for j, (w, b, stride) in enumerate(self.ha_w):
            last = j == len(self.ha_w) - 1
            out = self.Z if last else self.ha_buf[j]
            cout = w.shape[0]
            ops.conv3x3(x, cin, cin, B, H, H, w, b, out, cout, cout, dt, stride=stride,
                        act=ops.ACT_NONE if last else ops.ACT_GELU)
            H = (H + 2 - 3) // stride + 1
            x, cin = out, cout
        return shuf, rest

    def _back(self, shuf, in_chans):
        """g_s + decoder + unpatchify (MCM.py:636-688, 790-797) from YH; returns x_hat NCHW f32"""
        m, dt, B = self.m, self.dtype, self.batch
        Dd, K, L, P = m.decoder_embed_dim, m.num_keep_patches, self.L, self.P
        Td = L + 1
        # ---- g_s (MCM.py:790-792): transposed 1x1 convs back to E-dim tokens
        x = self.YH
        for j, (w, b) in enumerate(self.gs_w):
            last = j == len(self.gs_w) - 1
            ops.linear(x, w, b, dt, act=ops.ACT_NONE if last else ops.ACT_GELU, out=self.gs_buf[j])
            x = self.gs_buf[j]

        # ---- decoder (MCM.py:636-688): embed + unshuffle (+ off-by-one cls), blocks, norm, pred+unpatchify
        pos_d = m.decoder_pos_embed.detach()
        ops.decoder_embed(x, self.w_de, m.decoder_embed.bias.detach(), pos_d, shuf, self.dec, B, K, L, dt)
        ops.mask_rows(self.dec, m.mask_token.detach(), pos_d, shuf, B, L, K, Dd)
        for w in self.dec_w:
            run_block(self.dec, w, B, Td, dt, self.dec_s)
        ops.layernorm(self.dec, m.decoder_norm.weight, m.decoder_norm.bias, m.decoder_norm.eps, dt, rows=B * L,
                      row_group=L, group_stride=Td, row_offset=1, out=self.dn)
        x_hat = torch.empty((B, in_chans, self.img, self.img), dtype=torch.float32, device=self.device)
        ops.decoder_pred(self.dn, self.w_dp, self.b_dp, x_hat, B, L, P, dt, channel_planar=self.pred_cp)
        return x_hat

    # ------------------------------------------------------------------ Gaussian-conditional slice steps
    # Each is called with (i0, nbs, mu, sigma, ms_stride): slices i0..i0+nbs-1, mu/sigma device addresses
    # of rows [Mp][sw] per slice, ms_stride elements apart; it must leave y_hat (pre-LRP) in SUPY (operand
    # dtype) and YPRE (f32) at channels i0*sw.. .
    def _gc_forward(self, y_noise):
        M, sw, B, HW, dt = self.m.latent_depth, self.sw, self.batch, self.g * self.g, self.dtype

        def step(i0, nbs, mu, sigma, ms_stride):
            ops.gc_slices(self.Y32, M, i0 * sw, mu, sigma, ms_stride, sw, y_noise, self.YLIK, M, self.SUPY, dt, M,
                          self.YPRE, M, B, HW, nbs, sw)
        return step

    def _gc_compress(self, sym, idx):
        """eval step + int32 symbols / scale indexes in the coder's [slice][image][channel][pixel] order"""
        M, sw, B, HW, dt = self.m.latent_depth, self.sw, self.batch, self.g * self.g, self.dtype
        table = self.m.gaussian_conditional.scale_table
        per = B * sw * HW

        def step(i0, nbs, mu, sigma, ms_stride):
            ops.gc_slices_code(self.Y32, M, i0 * sw, mu, sigma, ms_stride, sw, self.YLIK, M, self.SUPY, dt, M,
                               self.YPRE, M, B, HW, nbs, sw, sym[i0 * per:], idx[i0 * per:], table)
        return step

    def _gc_decompress(self, decoder):
        """indexes on the device -> host rANS decode of the next slices' symbols -> y_hat = symbols + mu"""
        gc = self.m.gaussian_conditional
        M, sw, B, HW, dt = self.m.latent_depth, self.sw, self.batch, self.g * self.g, self.dtype
        cdf, sizes, offsets = gc.host_tables()
        bound = float(gc.scale_bound) if gc.scale_bound is not None else 0.11
        per = B * sw * HW
        idx_dev = torch.empty(self.m.num_slices * per, dtype=torch.int32, device=self.device)

        def step(i0, nbs, mu, sigma, ms_stride):
            n = nbs * per
            ops.gc_indexes(sigma, ms_stride, sw, B, HW, nbs, sw, gc.scale_table, bound, idx_dev)
            idx = idx_dev[:n].cpu().numpy()
            vals = decoder.decode_stream_array(idx, cdf, sizes, offsets)
            sym = torch.from_numpy(vals).to(self.device)
            ops.gc_dequantize(sym, mu, ms_stride, sw, B, HW, nbs, sw, i0 * sw, self.SUPY, dt, M, self.YPRE, M)
        return step

    def _h_s(self):
        """h_s_scale -> LS and h_s_mean -> LM (MCM.py:747-748): both stacks have the same shapes and read
        the same z_hat, so every layer is ONE launch of 2 problems ([scale, mean] weight / output slabs)"""
        B, dt = self.batch, self.dtype
        x, xs, cin, H = self.ZHAT, 0, self.m.hyperprior_depth, self.hz
        for j, (w, b, pshuf) in enumerate(self.hs2_w):
            last = j == len(self.hs2_w) - 1
            cout = w.shape[1]
            out = self.LSM if last else self.hs_buf[j]
            ops.conv3x3(x, cin, cin, B, H, H, w, b, out, out.shape[2], cout, dt,
                        act=ops.ACT_NONE if last else ops.ACT_GELU, pixel_shuffle=pshuf, nb=(1, 2),
                        strides={"x1": (0, xs), "w": (0, w[0].numel()), "b": (0, cout), "y": (0, out[0].numel())})
            if pshuf:
                H *= 2
                cin = cout // 4
            else:
                cin = cout
            x, xs = out, out[0].numel()

    def _slices(self, gc_step, chain_ok=False):
        m, dt, B, g = self.m, self.dtype, self.batch, self.g
        M, S, sw, ms, nb, Mp = m.latent_depth, m.num_slices, self.sw, self.maxsup, self.nb, self.Mp
        mid = self.mid
        c0 = mid[0]
        Pw = self.PW
        Pb = self.Pbuf
        eP = Pb.element_size()
        pbase = Pb.data_ptr()
        off_mean, off_lrp, off_scale = 0, S * c0, 2 * S * c0
        esz = self.SUPY.element_size()
        supy, ypre, yh = self.SUPY.data_ptr(), self.YPRE.data_ptr(), self.YH.data_ptr()
        e4 = 4
        # latent-channel partial sums of the first convs of slices [i0, i1): mean + lrp (one 2-problem launch
        # on LM, weight / output slabs S*c0 apart) and scale (on LS)
        wrow = self.w_pre_ml[0].numel()

        def pre(i0, i1):
            if self.w_lat is not None:  # every stack's block of slices [i0, i1) in one launch
                nfs = c0 // 16
                ops.lic_latent(B, g, [self.LM, self.LM, self.LS], M, M, self.w_lat, nfs, self.w_lat[0].numel(),
                               [0, S * nfs, 2 * S * nfs], i0 * nfs, i1 * nfs, pbase, Pw)
                return
            n = (i1 - i0) * c0
            ops.conv3x3(self.LM, M, M, B, g, g, self.w_pre_ml[i0 * c0:], None, pbase + (off_mean + i0 * c0) * eP, Pw,
                        n, dt, y_f32=True, nb=(1, 2), strides={"w": (0, S * c0 * wrow), "y": (0, S * c0)})
            ops.conv3x3(self.LS, M, M, B, g, g, self.w_pre_s[i0 * c0:], None, pbase + (off_scale + i0 * c0) * eP,
                        Pw, n, dt, y_f32=True)

        # The serial slice steps run 64-256-workgroup launches that leave most CUs idle: the partial sums of
        # slices 1.. are computed on a side stream under them (fork / join by events, graph-capturable);
        # slice i's first conv waits only for its own group.  Slice 0's group runs first on the main stream.
        ready = {}
        groups = [(i, i + 1) for i in range(1, ms)] + ([(ms, S)] if nb > 0 else [])
        if self.overlap and groups:
            main = torch.cuda.current_stream()
            pre(0, 1)
            fork = torch.cuda.Event()
            fork.record(main)
            side = self.side_stream
            side.wait_event(fork)
            with torch.cuda.stream(side):
                for i0, i1 in groups:
                    pre(i0, i1)
                    ev = torch.cuda.Event()
                    ev.record(side)
                    ready[i0] = ev
        else:
            pre(0, S)

        def wait_pre(i0):
            if i0 in ready:
                torch.cuda.current_stream().wait_event(ready.pop(i0))

        cm = [t.data_ptr() for t in self.CM]
        cl = [t.data_ptr() for t in self.CL]
        musig = self.MUSIG.data_ptr()
        cm_s1 = [nb * Mp * c for c in mid[:-1]]
        ms_s1 = nb * Mp * sw

        def ms_stack(first, layers, x1, c1, i0, nbs):
            """mean+scale stacks for slices i0.. (nbs problems per type) -> MUSIG"""
            w, b = first
            ops.conv3x3(x1, c1, M, B, g, g, w, b, cm[0], c0, c0, dt, act=ops.ACT_GELU,
                        addend=pbase + (off_mean + i0 * c0) * eP, ld_add=Pw, nb=(2, nbs),
                        strides={"w": (w[0].numel(), w[0][0].numel() if nbs > 1 else 0),
                                 "b": (b[0].numel(), c0 if nbs > 1 else 0),
                                 "a": (off_scale - off_mean, c0), "y": (cm_s1[0], Mp * c0)})
            for j, (w, b) in enumerate(layers):
                cin, cout = mid[j], mid[j + 1]
                last = j == len(layers) - 1
                y = musig if last else cm[j + 1]
                ys1 = ms_s1 if last else cm_s1[j + 1]
                ops.conv3x3(cm[j], cin, cin, B, g, g, w, b, y, cout, cout, dt,
                            act=ops.ACT_NONE if last else ops.ACT_GELU, y_f32=last, nb=(2, nbs),
                            strides={"x1": (cm_s1[j], Mp * cin), "w": (w[0].numel(), w[0][0].numel() if nbs > 1 else 0),
                                     "b": (b[0].numel(), cout if nbs > 1 else 0), "y": (ys1, Mp * cout)})

        def ms_fused(i0, nbs):
            """mean+scale stacks of slices i0.. as ONE tmae_lic_stack launch (2 x nbs problems) -> MUSIG"""
            ws = self.lstk["b_ms"] if nbs > 1 else self.lstk["ms"][i0]
            first, layers = (self.b_ms_first, self.b_ms_layers) if nbs > 1 else (self.ms_first[i0], self.ms_layers[i0])
            bs_ = [first[1]] + [b for _, b in layers]
            st = {"a": (off_scale - off_mean, c0), "y": (ms_s1, Mp * sw)}
            for l, (w, b) in enumerate(zip(ws, bs_)):
                st[f"w{l}"] = (w[0].numel(), w[0][0].numel() if nbs > 1 else 0)
                st[f"b{l}"] = (b[0].numel(), b.shape[-1] if nbs > 1 else 0)
            ops.lic_stack(B, g, supy, sw * (ms if nbs > 1 else i0), M, ws, bs_, mid, musig, sw, True,
                          addend=pbase + (off_mean + i0 * c0) * eP, ld_add=Pw, nb=(2, nbs), strides=st)

        def lrp_fused(i0, nbs):
            """lrp stack(s) of slices i0.. as one tmae_lic_stack launch: y_hat = y_hat_pre + 0.5 tanh(lrp) -> YH"""
            ws = self.lstk["b_lrp"] if nbs > 1 else self.lstk["lrp"][i0]
            first, layers = (self.b_lrp_first, self.b_lrp_layers) if nbs > 1 else (self.lrp_first[i0], self.lrp_layers[i0])
            bs_ = [first[1]] + [b for _, b in layers]
            st = {"a": (0, c0), "y": (0, sw), "src": (0, sw), "x2": (0, sw)}
            for l, (w, b) in enumerate(zip(ws, bs_)):
                st[f"w{l}"] = (0, w[0].numel() if nbs > 1 else 0)
                st[f"b{l}"] = (0, b.shape[-1] if nbs > 1 else 0)
            if nbs > 1:  # shared slots 0..ms-1 + own pre-LRP slot
                x = dict(x2=supy + ms * sw * esz, c2=sw, ld2=M)
                c1 = sw * ms
            else:        # y_hat slots 0..i0 (contiguous); also the support slot
                x = dict(y2=supy + i0 * sw * esz, ldy2=M)
                c1 = sw * (i0 + 1)
            ops.lic_stack(B, g, supy, c1, M, ws, bs_, mid, yh + i0 * sw * esz, M, False,
                          addend=pbase + (off_lrp + i0 * c0) * eP, ld_add=Pw, lrp_src=ypre + i0 * sw * e4, ld_src=M,
                          nb=(1, nbs), strides=st, **x)

        def lrp_stack(first, layers, i0, nbs, x2=None):
            w, b = first
            if x2 is None:  # single slice i0: input = y_hat slots 0..i0 (contiguous)
                ops.conv3x3(supy, sw * (i0 + 1), M, B, g, g, w, b, cl[0], c0, c0, dt, act=ops.ACT_GELU,
                            addend=pbase + (off_lrp + i0 * c0) * eP, ld_add=Pw)
            else:           # batched slices: shared slots 0..ms-1 + own pre-LRP slot
                ops.conv3x3(supy, sw * ms, M, B, g, g, w, b, cl[0], c0, c0, dt, act=ops.ACT_GELU,
                            x2=x2, c2=sw, ld2=M, addend=pbase + (off_lrp + i0 * c0) * eP, ld_add=Pw, nb=(1, nbs),
                            strides={"x2": (0, sw), "w": (0, w[0].numel()), "b": (0, c0), "a": (0, c0),
                                     "y": (0, Mp * c0)})
            for j, (w, b) in enumerate(layers):
                cin, cout = mid[j], mid[j + 1]
                if j < len(layers) - 1:
                    ops.conv3x3(cl[j], cin, cin, B, g, g, w, b, cl[j + 1], cout, cout, dt, act=ops.ACT_GELU,
                                nb=(1, nbs), strides={"x1": (0, Mp * cin), "w": (0, w[0].numel() if nbs > 1 else 0),
                                                      "b": (0, cout if nbs > 1 else 0), "y": (0, Mp * cout)})
                else:  # y_hat = y_hat_pre + 0.5 tanh(lrp) -> YH (and the support slot for i < ms)
                    ops.conv3x3(cl[j], cin, cin, B, g, g, w, b, yh + i0 * sw * esz, M, cout, dt,
                                y_f32=(dt == torch.float32), lrp_src=ypre + i0 * sw * e4, ld_src=M,
                                y2=(supy + i0 * sw * esz) if nbs == 1 else None, ldy2=M, nb=(1, nbs),
                                strides={"x1": (0, Mp * cin), "w": (0, w[0].numel() if nbs > 1 else 0),
                                         "b": (0, cout if nbs > 1 else 0), "src": (0, sw), "y": (0, sw),
                                         "y2": (0, sw)})

        # slices 0..ms-1: serial (slice i conditions on y_hat 0..i-1)
        fused = self.lstk is not None
        # serial slices as ONE launch each: the mean stack's workgroups go on with the slice's lrp stack
        # (y_hat_pre = round(y - mu) + mu in between), the scale stacks run beside them; the slices' Gaussian
        # likelihoods follow the loop in one launch (nothing in the chain reads them)
        chain = fused and chain_ok and self.USE_LIC_CHAIN
        ms_ser = self.MS_SER.data_ptr()
        yv = self.Y32.data_ptr()

        def ms_chain(i):
            ws, (first, layers) = self.lstk["ms"][i], (self.ms_first[i], self.ms_layers[i])
            bs_ = [first[1]] + [b for _, b in layers]
            st = {"a": (off_scale - off_mean, c0), "y": (S * Mp * sw, 0)}
            for l, (w, b) in enumerate(zip(ws, bs_)):
                st[f"w{l}"] = (w[0].numel(), 0)
                st[f"b{l}"] = (b[0].numel(), 0)
            lw = self.lstk["lrp"][i]
            lb_ = [self.lrp_first[i][1]] + [b for _, b in self.lrp_layers[i]]
            ch = dict(w=lw, b=lb_, couts=mid, x1=supy, c1=sw * i, ld1=M, y=yv + i * sw * e4, ldy=M,
                      add=pbase + (off_lrp + i * c0) * eP, ld_add=Pw, ypre=ypre + i * sw * e4, ld_ypre=M,
                      out=yh + i * sw * esz, ld_out=M, out2=supy + i * sw * esz, ld_out2=M)
            ops.lic_stack(B, g, supy, sw * i, M, ws, bs_, mid, ms_ser + i * Mp * sw * e4, sw, True,
                          addend=pbase + (off_mean + i * c0) * eP, ld_add=Pw, nb=(2, 1), strides=st, chain=ch)

        for i in range(ms):
            wait_pre(i)
            if chain:
                ms_chain(i)
                continue
            if fused:
                ms_fused(i, 1)
            else:
                ms_stack(self.ms_first[i], self.ms_layers[i], supy, sw * i, i, 1)
            gc_step(i, 1, musig, musig + ms_s1 * e4, Mp * sw)
            if fused:
                lrp_fused(i, 1)
            else:
                lrp_stack(self.lrp_first[i], self.lrp_layers[i], i, 1)
        # slices ms..S-1: batched on the fixed support y_hat 0..ms-1 (chaining them into their lrp stacks as
        # well measured slower, round 3)
        if nb > 0:
            wait_pre(ms)
            if fused:
                ms_fused(ms, nb)
            else:
                ms_stack(self.b_ms_first, self.b_ms_layers, supy, sw * ms, ms, nb)
            gc_step(ms, nb, musig, musig + ms_s1 * e4, Mp * sw)
            if fused:
                lrp_fused(ms, nb)
            else:
                lrp_stack(self.b_lrp_first, self.b_lrp_layers, ms, nb, x2=supy + ms * sw * esz)
        if chain:  # likelihoods of the chained slices (overwrites their dead SUPY / YPRE slots)
            gc_step(0, ms, ms_ser, ms_ser + S * Mp * sw * e4, Mp * sw)
        for k in list(ready):  # join the side stream in every case
            wait_pre(k)
