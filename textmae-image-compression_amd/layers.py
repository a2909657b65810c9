"""Parameter containers with the reference's third-party module names, so reference state_dicts load
unchanged and ``named_parameters()`` matches what ``configure_optimizers`` splits on.

* timm 0.4.5 ``PatchEmbed`` / ``Attention`` / ``Mlp`` / ``Block`` (used at reference
  models/Compression/MCM.py:300-348) — construction order and init identical, so a given
  ``torch.manual_seed`` produces the reference's initial weights;
* compressai 1.2.4 ``conv3x3`` / ``subpel_conv3x3`` (MCM.py:115-162).

Their ``forward`` methods run the HIP kernels (f32 parity path, or bf16 when the module's
``compute_dtype`` is set); MCM drives the same kernels through its own executor with persistent
workspaces.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops


def _pair(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


class PatchEmbed(nn.Module):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.img_size = _pair(img_size)
        self.patch_size = _pair(patch_size)
        self.num_patches = (self.img_size[1] // self.patch_size[1]) * (self.img_size[0] // self.patch_size[0])
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=self.patch_size, stride=self.patch_size)


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)


class Attention(nn.Module):
    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.num_heads = num_heads
        self.scale = qk_scale or (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)


class Block(nn.Module):
    """Pre-LN ViT block: x += proj(attn(norm1(x))); x += fc2(gelu(fc1(norm2(x))))."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, qk_scale=None, drop=0.0, attn_drop=0.0,
                 drop_path=0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop,
                              proj_drop=drop)
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        self.compute_dtype = torch.float32

    @torch.no_grad()
    def forward(self, x):
        """x: [B, T, D] f32 on the GPU."""
        b, t, d = x.shape
        resid = x.float().contiguous().clone()
        w = BlockWeights.from_block(self, self.compute_dtype)
        run_block(resid, w, b, t, self.compute_dtype, BlockScratch(b * t, d, w.hidden, self.compute_dtype, x.device))
        return resid


# ------------------------------------------------------------------------------------ execution
class BlockWeights:
    """One Block's weights in kernel layout ([N][K] linear weights in the compute dtype, f32 biases)."""

    __slots__ = ("n1w", "n1b", "eps1", "qkv_w", "qkv_b", "proj_w", "proj_b", "n2w", "n2b", "eps2", "fc1_w", "fc1_b",
                 "fc2_w", "fc2_b", "heads", "scale", "dim", "hidden")

    @staticmethod
    def from_block(blk: Block, dtype):
        w = BlockWeights()
        cast = (lambda t: t.detach().contiguous()) if dtype == torch.float32 else (
            lambda t: t.detach().to(dtype).contiguous())
        w.n1w, w.n1b, w.eps1 = blk.norm1.weight.detach(), blk.norm1.bias.detach(), blk.norm1.eps
        w.n2w, w.n2b, w.eps2 = blk.norm2.weight.detach(), blk.norm2.bias.detach(), blk.norm2.eps
        w.qkv_w, w.qkv_b = cast(blk.attn.qkv.weight), _b(blk.attn.qkv.bias)
        w.proj_w, w.proj_b = cast(blk.attn.proj.weight), _b(blk.attn.proj.bias)
        w.fc1_w, w.fc1_b = cast(blk.mlp.fc1.weight), _b(blk.mlp.fc1.bias)
        w.fc2_w, w.fc2_b = cast(blk.mlp.fc2.weight), _b(blk.mlp.fc2.bias)
        w.heads, w.scale = blk.attn.num_heads, blk.attn.scale
        w.dim, w.hidden = blk.attn.qkv.in_features, blk.mlp.fc1.out_features
        return w


def _b(t):
    return None if t is None else t.detach()


class BlockScratch:
    def __init__(self, rows, dim, hidden, dtype, device):
        self.a = torch.empty((rows, dim), dtype=dtype, device=device)
        self.qkv = torch.empty((rows, 3 * dim), dtype=dtype, device=device)
        self.att = torch.empty((rows, dim), dtype=dtype, device=device)
        self.h = torch.empty((rows, hidden), dtype=dtype, device=device)


def run_block(resid, w: BlockWeights, B, T, dtype, s: BlockScratch):
    """timm Block forward on the f32 residual stream `resid` [B*T, D], in place (7 launches)."""
    rows = B * T
    ops.layernorm(resid, w.n1w, w.n1b, w.eps1, dtype, rows=rows, out=s.a)
    dh = w.dim // w.heads
    if w.qkv_b is not None and ops.qkv_attn_supported(T, w.heads, dh, dtype):
        # qkv Linear + attention in one launch: Q / K / V never leave the chip (csrc/qkv_attn.hip)
        ops.qkv_attn(s.a, w.qkv_w, w.qkv_b, B, T, w.heads, dh, w.scale, dtype, out=s.att)
    else:
        ops.linear(s.a, w.qkv_w, w.qkv_b, dtype, out=s.qkv)
        ops.mha(s.qkv, B, T, w.heads, dh, w.scale, dtype, out=s.att)
    ops.linear_residual(s.att, w.proj_w, w.proj_b, resid, dtype)
    ops.layernorm(resid, w.n2w, w.n2b, w.eps2, dtype, rows=rows, out=s.a)
    ops.linear(s.a, w.fc1_w, w.fc1_b, dtype, act=ops.ACT_GELU, out=s.h)
    ops.linear_residual(s.h, w.fc2_w, w.fc2_b, resid, dtype)


# ------------------------------------------------------------------------------------ compressai layers
def conv3x3(in_ch, out_ch, stride=1):
    return nn.Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def subpel_conv3x3(in_ch, out_ch, r=1):
    return nn.Sequential(nn.Conv2d(in_ch, out_ch * r ** 2, kernel_size=3, padding=1), nn.PixelShuffle(r))
