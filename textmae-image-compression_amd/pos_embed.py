"""Fixed 2-D sin-cos position tables (reference models/Compression/common/pos_embed.py:23-94):
half the channels encode the grid row, half the column; each half is [sin | cos] of
pos * 10000^(-2i/d), computed in float64 and stored as float32 with a zero cls row."""
from __future__ import annotations

import numpy as np


def _sincos_1d(dim: int, pos: np.ndarray) -> np.ndarray:
    assert dim % 2 == 0
    freq = 1.0 / 10000 ** (np.arange(dim // 2, dtype=np.float64) / (dim / 2.0))
    ang = pos.reshape(-1)[:, None] * freq[None, :]
    return np.concatenate([np.sin(ang), np.cos(ang)], axis=1)


def get_2d_sincos_pos_embed(embed_dim: int, grid_size: int, cls_token: bool = False) -> np.ndarray:
    coords = np.arange(grid_size, dtype=np.float32)
    gw, gh = np.meshgrid(coords, coords)  # w first, as in the reference
    emb = np.concatenate([_sincos_1d(embed_dim // 2, gw), _sincos_1d(embed_dim // 2, gh)], axis=1)
    if cls_token:
        emb = np.concatenate([np.zeros([1, embed_dim]), emb], axis=0)
    return emb


def interpolate_pos_embed(model, checkpoint_model) -> None:
    """Resample a checkpoint's ``pos_embed`` to the model's patch grid, in place (reference
    models/Compression/common/pos_embed.py:103-132, DeiT's recipe; called by training.py:173-174 when
    ``--checkpoint`` is given).  The leading extra tokens (cls) are kept; the square grid of position
    tokens is resized bicubically (align_corners=False) from the checkpoint's side to sqrt(num_patches).
    A one-time host-side checkpoint edit, not part of the device path: it runs on the checkpoint's
    tensors with torch's own bicubic kernel, so the result is bitwise the reference's
    (tests/golden/pos_interp.npz, made by the reference function)."""
    import torch

    if "pos_embed" not in checkpoint_model:
        return
    pe = checkpoint_model["pos_embed"]
    dim = pe.shape[-1]
    num_patches = model.encoder_embed.num_patches
    extra = model.encoder_pos_embed.shape[-2] - num_patches
    src = int((pe.shape[-2] - extra) ** 0.5)
    dst = int(num_patches ** 0.5)
    if src == dst:
        return
    grid = pe[:, extra:].reshape(-1, src, src, dim).permute(0, 3, 1, 2)
    grid = torch.nn.functional.interpolate(grid, size=(dst, dst), mode="bicubic", align_corners=False)
    checkpoint_model["pos_embed"] = torch.cat((pe[:, :extra], grid.permute(0, 2, 3, 1).flatten(1, 2)), dim=1)
