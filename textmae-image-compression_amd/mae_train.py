"""Training path of MaskedAutoencoderViT (reference models/MAE/models_mae.py:216-220 under autograd:
``loss, pred, mask = model(imgs, mask_ratio)``, ``loss.backward()``).

As for MCM (mcm_train.py), one ``torch.autograd.Function`` covers the model: its forward runs the inference
kernels while keeping what the backward needs (per-block LayerNorm outputs, GELU inputs, attention log-sum-exp,
the gathered kept patches); its backward is the reverse pass on HIP kernels writing every parameter gradient into
one flat f32 buffer whose views autograd adopts as ``p.grad``:

  forward_loss (198-214)         tmae_mae_loss_bwd: mask * 2 (pred - target) / (p*p*c * sum(mask)), norm_pix targets
  decoder_pred / decoder_norm    split-K TN weight gradient, transposed-weight data gradient, LayerNorm backward
  decoder blocks                 the timm Block backward shared with MCM (_VitTrainBase._block_bwd)
  decoder_embed + mask_token     unshuffle gather of the token gradients (172-190: the cls row stays first), the
                                 mask-token gradient summed over the masked positions
  norm, encoder blocks           LayerNorm over every token (cls included), Block backward
  patch_embed / cls_token        weight gradient over the kept patches (the conv16/s16 as a GEMM), column sums
pos_embed / decoder_pos_embed are fixed sin-cos tables (requires_grad=False in the reference) and get none.
"""
from __future__ import annotations

import torch

from . import ops
from . import train_ops as T
from .mcm_train import _SIDE_SLOT_DIV, _VitTrainBase, _Weights, _block_params


class MAETrainExec(_VitTrainBase):
    """Workspaces + saved activations of one MAE training forward for (batch, len_keep, dtype, device)."""

    def __init__(self, m, batch, keep, dtype, device):
        self.m, self.batch, self.keep, self.dtype, self.device = m, batch, keep, dtype, device
        self.w = _Weights(dtype)
        self.P = m.patch_embed.patch_size[0]
        self.L = m.patch_embed.num_patches
        C = m.patch_embed.proj.in_channels
        # patch rows of KP = C*P*P values; the GEMMs take 16-B rows, so ViT-H's patch 14 (588 values) runs on rows
        # padded to Kw = 592: zero-tailed gathered patches, a zero-tailed copy of the weight, and a [E][Kw] weight
        # gradient of which the first KP columns are the parameter's
        self.KP = C * self.P * self.P
        self.Kw = -(-self.KP // 8) * 8
        # decoder_pred's KP outputs are the K of its data gradient and the rows of its weight gradient: in bf16
        # (16-B GEMM rows) a KP that is not a multiple of 8 runs on zero-tailed Kw-wide copies (dec_bwd)
        self._wpe_pad = self._gpe_pad = None
        self._dp_pad = None
        self.enc_gen = self.dec_gen = 0  # forward counters: a split backward refuses activations a later forward replaced
        self._layout()

    def _grad_order(self):
        m = self.m
        out = [m.decoder_pred.weight, m.decoder_pred.bias, m.decoder_norm.weight, m.decoder_norm.bias]
        for blk in reversed(m.decoder_blocks):
            out += _block_params(blk)
        out += [m.decoder_embed.weight, m.decoder_embed.bias, m.mask_token, m.norm.weight, m.norm.bias]
        for blk in reversed(m.blocks):
            out += _block_params(blk)
        out += [m.patch_embed.proj.weight, m.patch_embed.proj.bias, m.cls_token]
        seen = {id(p) for p in out}
        missing = [n for n, p in m.named_parameters() if p.requires_grad and id(p) not in seen]
        if missing:
            raise RuntimeError(f"MAE training executor does not cover parameters {missing}")
        return out

    # ------------------------------------------------------------------ forward
    def forward(self, imgs, noise):
        """-> (loss 0-d f32, pred f32 [B*L, p*p*c], mask [B, L])"""
        lat, mask = self.forward_enc(imgs, noise)
        pred = self.forward_dec(lat)
        loss = ops.mae_loss(pred, self.imgs, self.rest, self.keep, self.P, self.m.norm_pix_loss)
        return loss, pred, mask

    def forward_enc(self, imgs, noise):
        """forward_encoder (models_mae.py:150-170): -> (latent [B*Te, E] in the compute dtype, mask [B, L]); keeps
        the encoder's activations and the shuffle for the backward"""
        m, dt, B, keep, W = self.m, self.dtype, self.batch, self.keep, self.w
        E = m.pos_embed.shape[-1]
        P, Te = self.P, keep + 1
        self.enc_gen += 1
        imgs = imgs.float().contiguous()
        if imgs.shape[2:] != tuple(m.patch_embed.img_size):
            raise ValueError(f"Input image size {tuple(imgs.shape[2:])} doesn't match model {m.patch_embed.img_size}")
        self.imgs = imgs
        self.w.refresh()
        shuf, rest, mask = ops.mae_masking(noise, keep)
        self.shuf, self.rest = shuf, rest
        # patch embed of the kept patches + pos, cls row (models_mae.py:150-170)
        pw = m.patch_embed.proj.weight
        pos = m.pos_embed.detach()
        tok = torch.empty((B * Te, E), dtype=torch.float32, device=self.device)
        self.patches = T.patch_gather(imgs, shuf, self._e(B * keep, self.Kw), keep, P, dt)
        wpe = W.nt(pw)
        if self.Kw != self.KP:  # patch 14: the weight rows zero-tailed to Kw like the patches
            if self._wpe_pad is None:
                self._wpe_pad = self._z(E, self.Kw, dtype=dt)
            self._wpe_pad[:, :self.KP].copy_(wpe)
            wpe = self._wpe_pad
        ops.patch_embed(imgs, shuf, wpe, m.patch_embed.proj.bias.detach(), pos, tok, keep, P, dt,
                        patches=self.patches)
        ops.cls_rows(tok, m.cls_token.detach(), pos, B, Te, E)
        self.enc = []
        for blk in m.blocks:
            tok = self._block_fwd(blk, tok, B, Te)
        self.tok_last = tok
        return ops.layernorm(tok, m.norm.weight, m.norm.bias, m.norm.eps, dt), mask

    def forward_dec(self, lat):
        """forward_decoder (models_mae.py:172-196) of lat [B*Te, E] (compute dtype) under self.shuf: embed every
        latent row, mask tokens, unshuffle, pos; blocks; norm; pred -> pred f32 [B*L, p*p*c]"""
        m, dt, B, keep, W = self.m, self.dtype, self.batch, self.keep, self.w
        Dd = m.decoder_pos_embed.shape[-1]
        L, Te = self.L, keep + 1
        self.dec_gen += 1
        self.w.refresh()  # (a no-op after forward_enc's)
        self.lat = lat
        shuf = self.shuf
        dpos = m.decoder_pos_embed.detach()
        dec = torch.empty((B * (L + 1), Dd), dtype=torch.float32, device=self.device)
        ops.decoder_embed(self.lat, W.nt(m.decoder_embed.weight), m.decoder_embed.bias.detach(), dpos, shuf, dec, B,
                          Te, L, dt)
        ops.mask_rows(dec, m.mask_token.detach(), dpos, shuf, B, L, Te, Dd)
        self.dec = []
        for blk in m.decoder_blocks:
            dec = self._block_fwd(blk, dec, B, L + 1, store=self.dec)
        self.dec_last = dec
        self.dn = ops.layernorm(dec, m.decoder_norm.weight, m.decoder_norm.bias, m.decoder_norm.eps, dt, rows=B * L,
                                row_group=L, group_stride=L + 1, row_offset=1)
        self.pred = ops.linear(self.dn, W.nt(m.decoder_pred.weight), m.decoder_pred.bias.detach(), dt,
                               out_dtype=torch.float32)
        return self.pred

    # ------------------------------------------------------------------ backward
    def backward(self, dloss, dpred, gflat, sync=None):
        self.bwd_begin(gflat, sync)
        m, B, L = self.m, self.batch, self.L
        # ---- forward_loss (models_mae.py:198-214)
        dl = dloss.float().contiguous().reshape(1) if dloss is not None else None
        dp_in = dpred.float().contiguous() if dpred is not None else None
        dP = T.mae_loss_bwd(self.pred, self.imgs, self.rest, self.keep, self.P, m.norm_pix_loss, dl, dp_in,
                            self._e(B * L, self.pred.shape[1]), self.dtype)
        self.enc_bwd(self.dec_bwd(dP))
        self._side_join()

    def bwd_begin(self, gflat, sync=None):
        self.gflat, self.sync = gflat, sync
        if sync is not None:
            sync.attach(gflat)
        self._side_begin()

    def dec_bwd(self, dP):
        """decoder backward from dP [B*L, p*p*c] (compute dtype): every decoder parameter's gradient; -> the
        gradient of the decoder's input latent, f32 [B*Te, E]"""
        m, dt, W, B, keep = self.m, self.dtype, self.w, self.batch, self.keep
        E, Dd = m.pos_embed.shape[-1], m.decoder_pos_embed.shape[-1]
        L, Te = self.L, keep + 1
        G = self.grad
        npred = self.pred.shape[1]
        # ---- decoder_pred (models_mae.py:193)
        ddn = torch.empty((B * L, Dd), dtype=torch.float32, device=self.device)
        if npred % 8 and dt != torch.float32:
            # bf16, patch 14 (588 outputs): the gradient and W^T zero-tailed to 592 columns (the tails stay zero), the
            # weight gradient [592][Dd] into a scratch whose first 588 rows are the parameter's
            npad = -(-npred // 8) * 8
            if self._dp_pad is None:
                self._dp_pad = self._z(B * L, npad, dtype=dt)
                self._wt_pad = self._z(Dd, npad, dtype=dt)
                self._gdp_pad = torch.empty((npad, Dd), dtype=torch.float32, device=self.device)
                self._gdb_pad = torch.empty(npad, dtype=torch.float32, device=self.device)
            self._dp_pad[:, :npred].copy_(dP)
            self._wt_pad[:, :npred].copy_(W.t(m.decoder_pred.weight))
            T.wgrad(self._dp_pad, self.dn, npad, Dd, B * L, self._gdp_pad, dt, bias=self._gdb_pad,
                    slot_div=_SIDE_SLOT_DIV)
            G(m.decoder_pred.weight).copy_(self._gdp_pad[:npred])
            G(m.decoder_pred.bias).copy_(self._gdb_pad[:npred])
            T.dgrad_linear(self._dp_pad, self._wt_pad, B * L, npad, Dd, dt, out=ddn)
        else:
            self._wg(dP, self.dn, npred, Dd, B * L, G(m.decoder_pred.weight), dt, bias=G(m.decoder_pred.bias))
            T.dgrad_linear(dP, W.t(m.decoder_pred.weight), B * L, npred, Dd, dt, out=ddn)
        # ---- decoder_norm (the cls row gets no gradient: pred drops it) + blocks
        ddec = self._z(B * (L + 1), Dd)
        ddec_op = ddec if dt == torch.float32 else self._z(B * (L + 1), Dd, dtype=dt)
        T.layernorm_bwd(self.dec_last, m.decoder_norm.weight, ddn, ddec, B * L, Dd, m.decoder_norm.eps,
                        G(m.decoder_norm.weight), G(m.decoder_norm.bias), dxop=None if dt == torch.float32 else ddec_op,
                        row_group=L, group_stride=L + 1, row_offset=1)
        self._ready(m.decoder_norm.bias)
        for blk, s in zip(reversed(m.decoder_blocks), reversed(self.dec)):
            ddec, ddec_op = self._block_bwd(blk, s, ddec, ddec_op, B, L + 1)
            self._ready(_block_params(blk)[-1])
        # ---- decoder_embed + mask tokens: row 0 of each image is the cls row, rows 1..keep the kept patches
        dtok = self._e(B * Te, Dd)
        T.decoder_embed_bwd_gather(ddec, self.shuf, dtok, B, Te, L, Dd, dt, dmask=G(m.mask_token).view(-1))
        self._wg(dtok, self.lat, Dd, E, B * Te, G(m.decoder_embed.weight), dt, bias=G(m.decoder_embed.bias))
        dlat = torch.empty((B * Te, E), dtype=torch.float32, device=self.device)
        T.dgrad_linear(dtok, W.t(m.decoder_embed.weight), B * Te, Dd, E, dt, out=dlat)
        self._ready(m.mask_token)
        return dlat

    def enc_bwd(self, dlat):
        """encoder backward from the latent's gradient dlat f32 [B*Te, E]: every encoder parameter's gradient"""
        m, dt, B, keep = self.m, self.dtype, self.batch, self.keep
        E, Te = m.pos_embed.shape[-1], keep + 1
        G = self.grad
        # ---- encoder norm (every row, cls included) + blocks
        dt_tok = self._z(B * Te, E)
        dt_op = dt_tok if dt == torch.float32 else self._z(B * Te, E, dtype=dt)
        T.layernorm_bwd(self.tok_last, m.norm.weight, dlat, dt_tok, B * Te, E, m.norm.eps, G(m.norm.weight),
                        G(m.norm.bias), dxop=None if dt == torch.float32 else dt_op)
        self._ready(m.norm.bias)
        for blk, s in zip(reversed(m.blocks), reversed(self.enc)):
            dt_tok, dt_op = self._block_bwd(blk, s, dt_tok, dt_op, B, Te)
            self._ready(_block_params(blk)[-1])
        # ---- patch embed (kept patches) + cls token
        pw = m.patch_embed.proj.weight
        if self.Kw == self.KP:
            self._wg(dt_op, self.patches, E, self.KP, B * keep, G(pw), dt, lda=E, a_remap=(keep, Te, 1))
        else:  # patch 14: [E][Kw] into a scratch (same split plan as the side stream's), its first KP columns kept
            if self._gpe_pad is None:
                self._gpe_pad = torch.empty((E, self.Kw), dtype=torch.float32, device=self.device)
            T.wgrad(dt_op, self.patches, E, self.Kw, B * keep, self._gpe_pad, dt, lda=E, a_remap=(keep, Te, 1),
                    slot_div=_SIDE_SLOT_DIV)
            T.relayout(self._gpe_pad, G(pw).view(E, self.KP), (E, self.KP), (self.Kw, 1))
        T.colsum(dt_tok, B * keep, E, G(m.patch_embed.proj.bias), row_group=keep, group_stride=Te, row_offset=1)
        T.colsum(dt_tok, B, E, G(m.cls_token).view(-1), row_group=1, group_stride=Te, row_offset=0)
        self._ready(m.cls_token)


class _MAETrainFn(torch.autograd.Function):
    """MaskedAutoencoderViT.forward as one autograd node: (imgs, *params) -> (loss, pred, mask)"""

    @staticmethod
    def forward(ctx, ex, noise, imgs, *params):
        loss, pred, mask = ex.forward(imgs, noise)
        ctx.ex, ctx.params = ex, params
        ctx.mark_non_differentiable(mask)
        return loss, pred, mask

    @staticmethod
    def backward(ctx, dloss, dpred, dmask):
        ex, params = ctx.ex, ctx.params
        fresh = any(p.grad is not None for p in params if p.requires_grad)
        gflat = ex.grads_buffer(fresh)
        sync = getattr(ex.m, "grad_sync", None)
        ex.backward(dloss, dpred, gflat, sync=sync)
        if sync is not None:
            sync.finish()
        out = []
        for p in params:
            if not p.requires_grad:
                out.append(None)
            else:
                off = ex.offsets[id(p)]
                out.append(gflat[off:off + p.numel()].view(p.shape))
        return (None, None, None, *out)


def train_forward(m, imgs, mask_ratio, noise):
    """MaskedAutoencoderViT.forward with autograd: (loss, pred [N, L, p*p*c], mask [N, L])"""
    imgs = imgs.float().contiguous()
    B = imgs.shape[0]
    keep = m._len_keep(mask_ratio)
    ex = getattr(m, "_train_exec", None)
    if ex is None or (ex.batch, ex.keep, ex.dtype, ex.device) != (B, keep, m.compute_dtype, imgs.device):
        ex = m._train_exec = MAETrainExec(m, B, keep, m.compute_dtype, imgs.device)
    if noise is None:
        noise = torch.rand(B, ex.L, device=imgs.device)
    params = [p for p in m.parameters()]
    loss, pred, mask = _MAETrainFn.apply(ex, noise.to(imgs.device).float().contiguous(), imgs, *params)
    return loss, pred.view(B, ex.L, -1), mask


# ---------------------------------------------------------------------- forward_encoder / forward_decoder alone
# (models_mae.py:150-196 as separate nn.Module calls under autograd: each is its own node over its own parameters;
# the executor keeps one set of activations per part, so a part's backward must come before that part's next
# forward -- checked by the executor's forward counters)
def _enc_params(m):
    out = [m.norm.weight, m.norm.bias]
    for blk in m.blocks:
        out += _block_params(blk)
    return out + [m.patch_embed.proj.weight, m.patch_embed.proj.bias, m.cls_token]


def _dec_params(m):
    out = [m.decoder_pred.weight, m.decoder_pred.bias, m.decoder_norm.weight, m.decoder_norm.bias,
           m.decoder_embed.weight, m.decoder_embed.bias, m.mask_token]
    for blk in m.decoder_blocks:
        out += _block_params(blk)
    return out


def _param_grads(ex, params, gflat):
    return [gflat[ex.offsets[id(p)]:ex.offsets[id(p)] + p.numel()].view(p.shape) if p.requires_grad else None
            for p in params]


class _MAEEncFn(torch.autograd.Function):
    """forward_encoder: (imgs, *encoder params) -> (latent f32 [B, Te, E], mask, ids_restore)"""

    @staticmethod
    def forward(ctx, ex, noise, imgs, *params):
        lat, mask = ex.forward_enc(imgs, noise)
        ctx.ex, ctx.params, ctx.gen = ex, params, ex.enc_gen
        ctx.mark_non_differentiable(mask, ex.rest)
        return lat.float().view(ex.batch, ex.keep + 1, -1), mask, ex.rest

    @staticmethod
    def backward(ctx, dlat, dmask, drest):
        ex, params = ctx.ex, ctx.params
        if ex.enc_gen != ctx.gen:
            raise RuntimeError("forward_encoder ran again on this model before this backward: its saved activations "
                               "are gone (backward each forward_encoder before the next)")
        gflat = ex.grads_buffer(any(p.grad is not None for p in params if p.requires_grad))
        ex.bwd_begin(gflat)
        ex.enc_bwd(dlat.float().contiguous().view(ex.batch * (ex.keep + 1), -1))
        ex._side_join()
        return (None, None, None, *_param_grads(ex, params, gflat))


class _MAEDecFn(torch.autograd.Function):
    """forward_decoder: (latent [B, Te, E], *decoder params) -> pred f32 [B, L, p*p*c] (ids_restore fixed)"""

    @staticmethod
    def forward(ctx, ex, ids_restore, x, *params):
        ex.rest = ids_restore
        ex.shuf = ops.invert_permutation(ids_restore)
        lat = x.reshape(ex.batch * (ex.keep + 1), -1).to(ex.dtype).contiguous()
        pred = ex.forward_dec(lat)
        ctx.ex, ctx.params, ctx.gen, ctx.xshape = ex, params, ex.dec_gen, x.shape
        return pred.view(ex.batch, ex.L, -1)

    @staticmethod
    def backward(ctx, dpred):
        ex, params = ctx.ex, ctx.params
        if ex.dec_gen != ctx.gen:
            raise RuntimeError("forward_decoder ran again on this model before this backward: its saved activations "
                               "are gone (backward each forward_decoder before the next)")
        gflat = ex.grads_buffer(any(p.grad is not None for p in params if p.requires_grad))
        ex.bwd_begin(gflat)
        dP = ex._e(ex.batch * ex.L, ex.pred.shape[1])
        dP.copy_(dpred.reshape(dP.shape))
        dlat = ex.dec_bwd(dP)
        ex._side_join()
        return (None, None, dlat.view(ctx.xshape), *_param_grads(ex, params, gflat))


def _exec_for(m, B, keep, device):
    ex = getattr(m, "_train_exec", None)
    if ex is None or (ex.batch, ex.keep, ex.dtype, ex.device) != (B, keep, m.compute_dtype, device):
        ex = m._train_exec = MAETrainExec(m, B, keep, m.compute_dtype, device)
    return ex


def train_forward_encoder(m, imgs, mask_ratio, noise):
    """MaskedAutoencoderViT.forward_encoder with autograd: (latent f32 [N, 1 + len_keep, E], mask, ids_restore)"""
    imgs = imgs.float().contiguous()
    ex = _exec_for(m, imgs.shape[0], m._len_keep(mask_ratio), imgs.device)
    if noise is None:
        noise = torch.rand(imgs.shape[0], ex.L, device=imgs.device)
    return _MAEEncFn.apply(ex, noise.to(imgs.device).float().contiguous(), imgs, *_enc_params(m))


def train_forward_decoder(m, x, ids_restore):
    """MaskedAutoencoderViT.forward_decoder with autograd: pred f32 [N, L, p*p*c] (gradients to x and the
    decoder's parameters)"""
    n, t, _ = x.shape
    ex = _exec_for(m, n, t - 1, x.device)
    return _MAEDecFn.apply(ex, ids_restore.to(x.device).to(torch.int64).contiguous(), x, *_dec_params(m))
