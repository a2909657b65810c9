"""MaskedAutoencoderViT -- drop-in for reference models/MAE/models_mae.py:22-220 (plus the factories
at 223-250), on the same MI355X kernels as the MCM path.

Same constructor, parameter names (``patch_embed, cls_token, pos_embed, blocks, norm, decoder_embed,
mask_token, decoder_pos_embed, decoder_blocks, decoder_norm, decoder_pred``), registration and
initialisation order as the reference, so seeded construction gives the reference's weights and
checkpoints load unchanged.  ``forward(imgs, mask_ratio)`` returns ``(loss, pred, mask)``.

Differences from the reference are MI355X execution details only:
  * ``noise=`` may be passed to forward / random_masking: the reference draws
    ``torch.rand(N, L, device=x.device)`` inside random_masking (models_mae.py:132); passing the same
    tensor reproduces its masks (the device default draws on the model's device, as the reference does).
  * ``compute_dtype``: torch.float32 (exact-f32 MFMA) or torch.bfloat16.
"""
from __future__ import annotations

from functools import partial

import torch
import torch.nn as nn

from . import ops
from .layers import Block, BlockScratch, BlockWeights, PatchEmbed, run_block
from .pos_embed import get_2d_sincos_pos_embed


class MaskedAutoencoderViT(nn.Module):
    """Masked Autoencoder with VisionTransformer backbone (models_mae.py:22)."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=1024, depth=24, num_heads=16,
                 decoder_embed_dim=512, decoder_depth=8, decoder_num_heads=16, mlp_ratio=4.0, norm_layer=nn.LayerNorm,
                 norm_pix_loss=False):
        super().__init__()
        # MAE encoder (models_mae.py:31-41)
        self.patch_embed = PatchEmbed(img_size, patch_size, in_chans, embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, embed_dim), requires_grad=False)
        self.blocks = nn.ModuleList([Block(embed_dim, num_heads, mlp_ratio, qkv_bias=True, qk_scale=None,
                                           norm_layer=norm_layer) for _ in range(depth)])
        self.norm = norm_layer(embed_dim)
        # MAE decoder (models_mae.py:45-58)
        self.decoder_embed = nn.Linear(embed_dim, decoder_embed_dim, bias=True)
        self.mask_token = nn.Parameter(torch.zeros(1, 1, decoder_embed_dim))
        self.decoder_pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, decoder_embed_dim), requires_grad=False)
        self.decoder_blocks = nn.ModuleList([Block(decoder_embed_dim, decoder_num_heads, mlp_ratio, qkv_bias=True,
                                                   qk_scale=None, norm_layer=norm_layer)
                                             for _ in range(decoder_depth)])
        self.decoder_norm = norm_layer(decoder_embed_dim)
        self.decoder_pred = nn.Linear(decoder_embed_dim, patch_size ** 2 * in_chans, bias=True)
        self.norm_pix_loss = norm_pix_loss
        self.initialize_weights()

        # MI355X execution settings (not part of the reference surface)
        self.compute_dtype = torch.float32
        self._exec = None
        self._train_exec = None

    # ---------------------------------------------------------------------------------- init
    def initialize_weights(self):
        """models_mae.py:62-81"""
        g = int(self.patch_embed.num_patches ** 0.5)
        self.pos_embed.data.copy_(torch.from_numpy(get_2d_sincos_pos_embed(self.pos_embed.shape[-1], g, True))
                                  .float().unsqueeze(0))
        self.decoder_pos_embed.data.copy_(
            torch.from_numpy(get_2d_sincos_pos_embed(self.decoder_pos_embed.shape[-1], g, True)).float().unsqueeze(0))
        w = self.patch_embed.proj.weight.data
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
        r = super().load_state_dict(state_dict, strict=strict)
        self._exec = None
        return r

    # ---------------------------------------------------------------------------------- layout helpers
    def patchify(self, imgs):
        """models_mae.py:86-98 (nchpwq -> nhwpqc)"""
        p = self.patch_embed.patch_size[0]
        assert imgs.shape[2] == imgs.shape[3] and imgs.shape[2] % p == 0
        h = w = imgs.shape[2] // p
        x = imgs.reshape(imgs.shape[0], 3, h, p, w, p)
        return torch.einsum("nchpwq->nhwpqc", x).reshape(imgs.shape[0], h * w, p ** 2 * 3)

    def unpatchify(self, x):
        p = self.patch_embed.patch_size[0]
        h = w = int(x.shape[1] ** 0.5)
        assert h * w == x.shape[1]
        x = torch.einsum("nhwpqc->nchpwq", x.reshape(x.shape[0], h, w, p, p, 3))
        return x.reshape(x.shape[0], 3, h * p, h * p)

    # ---------------------------------------------------------------------------------- execution
    def _check(self, imgs):
        if not imgs.is_cuda:
            raise ValueError("MaskedAutoencoderViT runs on the MI355X kernels: move the model and inputs to the GPU")

    def _training_call(self):
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    def _check_supported(self):
        """what the kernels cover: head dims 32 / 64 / 80 (attention)"""
        bad = []
        for name, blocks in (("encoder", self.blocks), ("decoder", self.decoder_blocks)):
            for b in blocks[:1]:
                dh = b.attn.qkv.in_features // b.attn.num_heads
                if dh not in (32, 64, 80):
                    bad.append(f"{name} head dim {dh} (32, 64 or 80 supported)")
        if bad:
            raise ValueError("MaskedAutoencoderViT configuration not supported by the MI355X kernels: " + "; ".join(bad))

    def _executor(self, batch, keep, device):
        self._check_supported()
        ex = self._exec
        if ex is None or (ex.batch, ex.keep, ex.dtype, ex.device) != (batch, keep, self.compute_dtype, device):
            ex = self._exec = _MAEExecutor(self, batch, keep, self.compute_dtype, device)
        ex.refresh_weights()
        return ex

    def _len_keep(self, mask_ratio):
        return int(self.patch_embed.num_patches * (1 - mask_ratio))

    def random_masking(self, x, mask_ratio, noise=None):
        """models_mae.py:123-148: (x_masked, mask, ids_restore); argsort on the device, stable."""
        N, L, D = x.shape
        len_keep = int(L * (1 - mask_ratio))
        if noise is None:
            noise = torch.rand(N, L, device=x.device)
        shuf, rest, mask = ops.mae_masking(noise.to(x.device), len_keep)
        x_masked = torch.gather(x, 1, shuf[:, :len_keep].unsqueeze(-1).repeat(1, 1, D))
        return x_masked, mask, rest

    def forward_encoder(self, x, mask_ratio, noise=None):
        """models_mae.py:150-170 -> (latent f32 [N, 1 + len_keep, E], mask, ids_restore); under autograd the
        training executor's encoder part (mae_train.py, HIP backward of the encoder)"""
        self._check(x)
        if self._training_call():
            self._check_supported()
            from .mae_train import train_forward_encoder

            return train_forward_encoder(self, x, mask_ratio, noise)
        with torch.no_grad():
            keep = self._len_keep(mask_ratio)
            ex = self._executor(x.shape[0], keep, x.device)
            _, rest, mask = ex.encode(x, noise, keep)
            return ex.latent_f32().view(x.shape[0], keep + 1, -1), mask, rest

    def forward_decoder(self, x, ids_restore):
        """models_mae.py:172-196 -> pred f32 [N, L, p*p*C]; under autograd (decoder parameters or x requiring
        gradients) the training executor's decoder part"""
        self._check(x)
        if self._training_call() or (torch.is_grad_enabled() and x.requires_grad):
            self._check_supported()
            from .mae_train import train_forward_decoder

            return train_forward_decoder(self, x, ids_restore)
        with torch.no_grad():
            n, t, _ = x.shape
            ex = self._executor(n, t - 1, x.device)
            shuf = ops.invert_permutation(ids_restore)
            return ex.decode(x.reshape(n * t, -1).contiguous(), shuf).view(n, self.patch_embed.num_patches, -1)

    def forward_loss(self, imgs, pred, mask):
        """models_mae.py:198-214 (torch ops: the forward path uses the fused tmae_mae_loss kernel)"""
        target = self.patchify(imgs)
        if self.norm_pix_loss:
            mean = target.mean(dim=-1, keepdim=True)
            var = target.var(dim=-1, keepdim=True)
            target = (target - mean) / (var + 1.0e-6) ** 0.5
        loss = ((pred - target) ** 2).mean(dim=-1)
        return (loss * mask).sum() / mask.sum()

    def forward(self, imgs, mask_ratio=0.75, noise=None):
        """models_mae.py:216-220 -> (loss, pred [N, L, p*p*3], mask [N, L]); under autograd the training path
        (mae_train.py: HIP backward of the whole model)"""
        self._check(imgs)
        if self._training_call():
            self._check_supported()
            from .mae_train import train_forward

            return train_forward(self, imgs, mask_ratio, noise)
        with torch.no_grad():
            imgs = imgs.float().contiguous()
            keep = self._len_keep(mask_ratio)
            ex = self._executor(imgs.shape[0], keep, imgs.device)
            shuf, rest, mask = ex.encode(imgs, noise, keep)
            pred = ex.decode(ex.lat, shuf)
            loss = ops.mae_loss(pred, imgs, rest, keep, self.patch_embed.patch_size[0], self.norm_pix_loss)
            return loss, pred.view(imgs.shape[0], self.patch_embed.num_patches, -1), mask


class _MAEExecutor:
    """Prepared weights + workspaces for one (batch, len_keep, dtype, device); graph-capturable."""

    def __init__(self, m: MaskedAutoencoderViT, batch, keep, dtype, device):
        self.m, self.batch, self.keep, self.dtype, self.device = m, batch, keep, dtype, device
        self._sig = None
        E, Dd = m.pos_embed.shape[-1], m.decoder_pos_embed.shape[-1]
        L = m.patch_embed.num_patches
        B, T = batch, keep + 1
        hid_e = m.blocks[0].mlp.fc1.out_features if len(m.blocks) else 4 * E
        hid_d = m.decoder_blocks[0].mlp.fc1.out_features if len(m.decoder_blocks) else 4 * Dd

        def z(*shape, dt=torch.float32):
            return torch.empty(shape, dtype=dt, device=device)

        self.tok = z(B * T, E)
        self.enc_s = BlockScratch(B * T, E, hid_e, dtype, device)
        self.lat = z(B * T, E, dt=dtype)
        self.dec = z(B * (L + 1), Dd)
        self.dec_s = BlockScratch(B * (L + 1), Dd, hid_d, dtype, device)
        self.dn = z(B * L, Dd, dt=dtype)

    def refresh_weights(self):
        sig = tuple((p.data_ptr(), p._version) for p in self.m.parameters())
        if sig == self._sig:
            return
        self._sig = sig
        m, dt = self.m, self.dtype
        cast = (lambda t: t.detach().contiguous()) if dt == torch.float32 else (
            lambda t: t.detach().to(dt).contiguous())
        w = m.patch_embed.proj.weight.detach()
        w = w.reshape(w.shape[0], -1)
        if w.shape[1] % 8:  # patch 14: rows of 588 values padded to 592 (tmae_patch_embed_fwd)
            w = torch.nn.functional.pad(w, (0, 8 - w.shape[1] % 8))
        self.w_pe = cast(w)
        self.enc_w = [BlockWeights.from_block(b, dt) for b in m.blocks]
        self.dec_w = [BlockWeights.from_block(b, dt) for b in m.decoder_blocks]
        self.w_de = cast(m.decoder_embed.weight)
        self.w_dp = cast(m.decoder_pred.weight)

    def encode(self, imgs, noise, keep):
        """patch embed (kept patches only) + pos, cls, blocks, norm -> self.lat; (ids_shuffle, ids_restore, mask)"""
        m, dt, B = self.m, self.dtype, self.batch
        E = m.pos_embed.shape[-1]
        L, P = m.patch_embed.num_patches, m.patch_embed.patch_size[0]
        T = keep + 1
        if imgs.shape[2:] != tuple(m.patch_embed.img_size):
            raise ValueError(f"Input image size {tuple(imgs.shape[2:])} doesn't match model {m.patch_embed.img_size}")
        if noise is None:
            noise = torch.rand(B, L, device=self.device)
        shuf, rest, mask = ops.mae_masking(noise.to(self.device), keep)
        pos = m.pos_embed.detach()
        ops.patch_embed(imgs.float().contiguous(), shuf, self.w_pe, m.patch_embed.proj.bias.detach(), pos, self.tok,
                        keep, P, dt)
        ops.cls_rows(self.tok, m.cls_token.detach(), pos, B, T, E)
        for w in self.enc_w:
            run_block(self.tok, w, B, T, dt, self.enc_s)
        ops.layernorm(self.tok, m.norm.weight, m.norm.bias, m.norm.eps, dt, out=self.lat)
        return shuf, rest, mask

    def latent_f32(self):
        m = self.m
        return ops.layernorm(self.tok, m.norm.weight, m.norm.bias, m.norm.eps, torch.float32)

    def decode(self, lat, shuf):
        """decoder_embed + mask tokens + unshuffle + pos (the cls row is the real cls here), blocks, norm,
        pred on the L patch rows -> f32 [B*L, p*p*C]"""
        m, dt, B, keep = self.m, self.dtype, self.batch, self.keep
        Dd = m.decoder_pos_embed.shape[-1]
        L = m.patch_embed.num_patches
        pos = m.decoder_pos_embed.detach()
        if lat.dtype != dt and lat.dtype != torch.float32:
            lat = lat.float()
        ops.decoder_embed(lat, self.w_de, m.decoder_embed.bias.detach(), pos, shuf, self.dec, B, keep + 1, L, dt)
        ops.mask_rows(self.dec, m.mask_token.detach(), pos, shuf, B, L, keep + 1, Dd)
        for w in self.dec_w:
            run_block(self.dec, w, B, L + 1, dt, self.dec_s)
        ops.layernorm(self.dec, m.decoder_norm.weight, m.decoder_norm.bias, m.decoder_norm.eps, dt, rows=B * L,
                      row_group=L, group_stride=L + 1, row_offset=1, out=self.dn)
        return ops.linear(self.dn, self.w_dp, m.decoder_pred.bias.detach(), dt, out_dtype=torch.float32)


def mae_vit_base_patch16_dec512d8b(**kwargs):
    """models_mae.py:223-228"""
    return MaskedAutoencoderViT(patch_size=16, embed_dim=768, depth=12, num_heads=12, decoder_embed_dim=512,
                                decoder_depth=8, decoder_num_heads=16, mlp_ratio=4,
                                norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


def mae_vit_large_patch16_dec512d8b(**kwargs):
    """models_mae.py:231-236"""
    return MaskedAutoencoderViT(patch_size=16, embed_dim=1024, depth=24, num_heads=16, decoder_embed_dim=512,
                                decoder_depth=8, decoder_num_heads=16, mlp_ratio=4,
                                norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


def mae_vit_huge_patch14_dec512d8b(**kwargs):
    """models_mae.py:239-244 (patch 14: per-value patch gather; head dim 80: attention tiles padded to 96)"""
    return MaskedAutoencoderViT(patch_size=14, embed_dim=1280, depth=32, num_heads=16, decoder_embed_dim=512,
                                decoder_depth=8, decoder_num_heads=16, mlp_ratio=4,
                                norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


# recommended arch names (models_mae.py:248-250)
mae_vit_base_patch16 = mae_vit_base_patch16_dec512d8b
mae_vit_large_patch16 = mae_vit_large_patch16_dec512d8b
mae_vit_huge_patch14 = mae_vit_huge_patch14_dec512d8b
