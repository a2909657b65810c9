"""TEST INFRASTRUCTURE ONLY -- CPU restatement (torch f32) of the reference MaskedAutoencoderViT
forward (models/MAE/models_mae.py:123-220; forward_encoder / forward_decoder as their own functions) on a plain state_dict, with timm 0.4.5's Block restated in
mcm_oracle.block.  Pinned against tests/golden/mae_forward.npz (made by the reference code itself).
Imported only by tests/.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .mcm_oracle import block, layer_norm, linear


def patchify(imgs, p):
    n, c, h, w = imgs.shape
    x = imgs.reshape(n, c, h // p, p, w // p, p)
    return torch.einsum("nchpwq->nhwpqc", x).reshape(n, (h // p) * (w // p), p * p * c)


def mae_encoder(sd, imgs, noise, mask_ratio, patch, heads, depth, eps=1e-6):
    """forward_encoder (models_mae.py:150-170) -> (latent [N, 1 + len_keep, D], mask [N, L], ids_restore)"""
    x = F.conv2d(imgs, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], stride=patch)
    x = x.flatten(2).transpose(1, 2)
    x = x + sd["pos_embed"][:, 1:, :]
    N, L, D = x.shape
    len_keep = int(L * (1 - mask_ratio))
    ids_shuffle = torch.argsort(noise, dim=1, stable=True)
    ids_restore = torch.argsort(ids_shuffle, dim=1, stable=True)
    ids_keep = ids_shuffle[:, :len_keep]
    x = torch.gather(x, 1, ids_keep.unsqueeze(-1).repeat(1, 1, D))
    mask = torch.ones([N, L])
    mask[:, :len_keep] = 0
    mask = torch.gather(mask, 1, ids_restore)
    cls = (sd["cls_token"] + sd["pos_embed"][:, :1, :]).expand(N, -1, -1)
    x = torch.cat((cls, x), dim=1)
    for i in range(depth):
        x = block(x, sd, f"blocks.{i}.", heads, eps)
    return layer_norm(x, sd, "norm.", eps), mask, ids_restore


def mae_decoder(sd, x, ids_restore, dec_heads, dec_depth, eps=1e-6):
    """forward_decoder (models_mae.py:172-196) -> pred [N, L, p*p*c]"""
    N, L = ids_restore.shape
    x = linear(x, sd, "decoder_embed.")
    mask_tokens = sd["mask_token"].repeat(N, L + 1 - x.shape[1], 1)
    x_ = torch.cat([x[:, 1:, :], mask_tokens], dim=1)
    x_ = torch.gather(x_, 1, ids_restore.unsqueeze(-1).repeat(1, 1, x.shape[2]))
    x = torch.cat([x[:, :1, :], x_], dim=1) + sd["decoder_pos_embed"]
    for i in range(dec_depth):
        x = block(x, sd, f"decoder_blocks.{i}.", dec_heads, eps)
    x = layer_norm(x, sd, "decoder_norm.", eps)
    return linear(x, sd, "decoder_pred.")[:, 1:, :]


def mae_forward(sd, imgs, noise, mask_ratio, patch, heads, dec_heads, depth, dec_depth, eps=1e-6, norm_pix=False):
    """-> (loss, pred [N, L, p*p*c], mask [N, L]) exactly as models_mae.forward with the given noise"""
    latent, mask, ids_restore = mae_encoder(sd, imgs, noise, mask_ratio, patch, heads, depth, eps)
    pred = mae_decoder(sd, latent, ids_restore, dec_heads, dec_depth, eps)
    target = patchify(imgs, patch)
    if norm_pix:
        mean = target.mean(dim=-1, keepdim=True)
        var = target.var(dim=-1, keepdim=True)
        target = (target - mean) / (var + 1.0e-6) ** 0.5
    loss = ((pred - target) ** 2).mean(dim=-1)
    return (loss * mask).sum() / mask.sum(), pred, mask
