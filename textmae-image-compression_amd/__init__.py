"""MI355X-native (gfx950) TextMAE MCM hot path: MAE-ViT encode/decode + entropy-bottleneck and
Gaussian-conditional rate estimation, behind the reference's nn.Module surface.

Import name: ``textmae_amd`` (see textmae_amd.py at the repo root; the directory name contains
dashes, as the build layout requires).
"""
from . import ops  # noqa: F401
from ._lib import LIB_PATH, load as load_library  # noqa: F401
from .entropy import CompressionModel, EntropyBottleneck, GaussianConditional, get_scale_table  # noqa: F401
from .layers import Block, PatchEmbed  # noqa: F401
from .mae import (MaskedAutoencoderViT, mae_vit_base_patch16, mae_vit_base_patch16_dec512d8b,  # noqa: F401
                  mae_vit_huge_patch14, mae_vit_huge_patch14_dec512d8b, mae_vit_large_patch16,
                  mae_vit_large_patch16_dec512d8b)
from .mcm import MCM  # noqa: F401
from .pos_embed import get_2d_sincos_pos_embed, interpolate_pos_embed  # noqa: F401

__all__ = ["MCM", "MaskedAutoencoderViT", "mae_vit_base_patch16_dec512d8b", "mae_vit_large_patch16_dec512d8b",
           "mae_vit_huge_patch14_dec512d8b", "Block", "PatchEmbed", "EntropyBottleneck", "GaussianConditional", "CompressionModel", "ops",
           "load_library", "LIB_PATH", "get_scale_table", "get_2d_sincos_pos_embed", "interpolate_pos_embed"]
