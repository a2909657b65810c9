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
