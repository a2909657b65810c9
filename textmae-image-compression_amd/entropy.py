"""Entropy models with compressai 1.2.4's parameter/buffer names and semantics, HIP-backed.

compressai is a third-party dependency of the reference (requirements.txt:9, used at
models/Compression/MCM.py:8-12, 71-72, 741-744, 771-776, utils/engine.py:79, testing.py:223); it
is not vendored and not installed here, so its published algorithm is restated (see DESIGN.md,
"parity unpinned" at that boundary).  Names match so reference checkpoints load unchanged:
``entropy_bottleneck.{_matrix0-4,_bias0-4,_factor0-3,quantiles,target,_offset,_quantized_cdf,
_cdf_length}``, ``gaussian_conditional.{scale_table,scale_bound,_offset,_quantized_cdf,_cdf_length}``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from . import ops


class LowerBound(nn.Module):
    """max(x, bound) (its custom backward lives with the training kernels)."""

    def __init__(self, bound):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return torch.max(x, self.bound.to(x.dtype))


class EntropyModel(nn.Module):
    def __init__(self, likelihood_bound=1e-9, entropy_coder=None, entropy_coder_precision=16):
        super().__init__()
        self.entropy_coder_precision = int(entropy_coder_precision)
        self.use_likelihood_bound = likelihood_bound > 0
        if self.use_likelihood_bound:
            self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())

    @property
    def offset(self):
        return self._offset

    @property
    def quantized_cdf(self):
        return self._quantized_cdf

    @property
    def cdf_length(self):
        return self._cdf_length


class EntropyBottleneck(EntropyModel):
    """Factorized prior: per-channel monotone MLP 1-3-3-3-3-1 density model."""

    def __init__(self, channels, *args, tail_mass=1e-9, init_scale=10, filters=(3, 3, 3, 3), **kwargs):
        super().__init__(*args, **kwargs)
        if tuple(filters) != (3, 3, 3, 3):
            raise NotImplementedError("the HIP entropy bottleneck implements compressai's default filters (3,3,3,3)")
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        filt = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        for i in range(len(self.filters) + 1):
            init = np.log(np.expm1(1 / scale / filt[i + 1]))
            matrix = torch.Tensor(channels, filt[i + 1], filt[i])
            matrix.data.fill_(init)
            self.register_parameter(f"_matrix{i:d}", nn.Parameter(matrix))
            bias = torch.Tensor(channels, filt[i + 1], 1)
            nn.init.uniform_(bias, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(bias))
            if i < len(self.filters):
                factor = torch.Tensor(channels, filt[i + 1], 1)
                nn.init.zeros_(factor)
                self.register_parameter(f"_factor{i:d}", nn.Parameter(factor))
        self.quantiles = nn.Parameter(torch.Tensor(channels, 1, 3))
        init = torch.Tensor([-self.init_scale, 0, self.init_scale])
        self.quantiles.data = init.repeat(self.quantiles.size(0), 1, 1)
        target = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _get_medians(self):
        return self.quantiles[:, :, 1:2]

    @torch.no_grad()
    def forward(self, x, training=None, noise=None):
        """x: NCHW f32 -> (outputs, likelihood), like compressai (outputs = x~ fed to the density)."""
        if training is None:
            training = self.training
        n, c, h, w = x.shape
        z = x.float().permute(0, 2, 3, 1).contiguous()
        if training and noise is None:
            noise = torch.empty_like(x, dtype=torch.float32).uniform_(-0.5, 0.5)
        lik, zhat = ops.eb_likelihood(self, z, n, c, h * w, noise=noise.contiguous() if training else None)
        outputs = (x.float() + noise) if training else zhat.view(n, h, w, c).permute(0, 3, 1, 2).contiguous()
        return outputs, lik.view(n, c, h, w)

    @torch.no_grad()
    def loss(self):
        return ops.eb_aux_loss(self)


class GaussianConditional(EntropyModel):
    def __init__(self, scale_table, *args, scale_bound=0.11, tail_mass=1e-9, **kwargs):
        super().__init__(*args, **kwargs)
        self.tail_mass = float(tail_mass)
        self.register_buffer("scale_table", torch.Tensor(tuple(float(s) for s in scale_table)) if scale_table
                             else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]) if scale_bound is not None else None)
        self.lower_bound_scale = LowerBound(scale_bound)

    @torch.no_grad()
    def forward(self, inputs, scales, means=None, training=None, noise=None):
        if training is None:
            training = self.training
        if training and noise is None:
            noise = torch.empty_like(inputs, dtype=torch.float32).uniform_(-0.5, 0.5)
        bound = float(self.scale_bound) if self.scale_bound is not None else 0.0
        return ops.gc_likelihood(inputs.float(), scales.float(), None if means is None else means.float(),
                                 noise if training else None, bound)


def get_scale_table(min_=0.11, max_=256, levels=64):
    """compressai.models.google.get_scale_table"""
    return torch.exp(torch.linspace(math.log(min_), math.log(max_), levels))


def _update_registered_buffers(module, module_name, buffer_names, state_dict):
    """compressai.models.utils.update_registered_buffers: resize empty buffers before loading."""
    valid = {n for n, _ in module.named_buffers()}
    for name in buffer_names:
        if name not in valid:
            continue
        key = f"{module_name}.{name}"
        if key in state_dict:
            new = state_dict[key]
            buf = getattr(module, name)
            if buf.numel() == 0 or buf.size() != new.size():
                getattr(module, name).resize_(new.size())


class CompressionModel(nn.Module):
    """compressai.models.CompressionModel surface: aux_loss(), update(), buffer-resizing load."""

    def __init__(self, entropy_bottleneck_channels=None, init_weights=None):
        super().__init__()

    def aux_loss(self):
        return sum(m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck))

    def load_state_dict(self, state_dict, strict=True):
        for name, module in self.named_modules():
            if not any(x.startswith(name) for x in state_dict.keys()):
                continue
            if isinstance(module, EntropyBottleneck):
                _update_registered_buffers(module, name, ["_quantized_cdf", "_offset", "_cdf_length"], state_dict)
            if isinstance(module, GaussianConditional):
                _update_registered_buffers(module, name, ["_quantized_cdf", "_offset", "_cdf_length", "scale_table"],
                                           state_dict)
        return nn.Module.load_state_dict(self, state_dict, strict=strict)
