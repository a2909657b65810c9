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

    def _check_cdf(self):
        if self._offset.numel() == 0 or self._quantized_cdf.numel() == 0 or self._cdf_length.numel() == 0:
            raise ValueError("Uninitialized CDFs. Run update() first")

    def _pmf_to_cdf(self, pmf, tail_mass, pmf_length, max_length):
        """EntropyModel._pmf_to_cdf: per row, pmf[:len] + tail -> quantized CDF (host C++ builder)"""
        from .coder import pmf_to_quantized_cdf

        pmf_h = pmf.detach().float().cpu().numpy()
        tail_h = tail_mass.detach().float().reshape(-1).cpu().numpy()
        lengths = pmf_length.detach().reshape(-1).cpu().tolist()
        cdf = torch.zeros((len(lengths), max_length + 2), dtype=torch.int32)
        for i, n in enumerate(lengths):
            prob = np.concatenate([pmf_h[i, :n], tail_h[i:i + 1]]).astype(np.float32)
            row = pmf_to_quantized_cdf(prob, self.entropy_coder_precision)
            cdf[i, :len(row)] = torch.tensor(row, dtype=torch.int32)
        return cdf.to(pmf.device)

    def host_tables(self):
        """(cdf int32 [n][len], cdf_length int32 [n], offset int32 [n]) as numpy, cached until the buffers change"""
        self._check_cdf()
        key = tuple((t.data_ptr(), t._version) for t in (self._quantized_cdf, self._cdf_length, self._offset))
        cache = getattr(self, "_host_tables_cache", None)
        if cache is None or cache[0] != key:
            tabs = tuple(np.ascontiguousarray(t.detach().cpu().numpy().astype(np.int32))
                         for t in (self._quantized_cdf, self._cdf_length.reshape(-1), self._offset.reshape(-1)))
            cache = (key, tabs)
            self._host_tables_cache = cache
        return cache[1]

    @staticmethod
    def quantize_symbols(inputs, means=None):
        """quantize(inputs, "symbols", means): round(inputs - means).int() (module-level convenience)"""
        x = inputs - means if means is not None else inputs
        return torch.round(x).int()

    @staticmethod
    def dequantize(inputs, means=None, dtype=torch.float):
        outputs = inputs.type(dtype)
        return outputs + means if means is not None else outputs

    def _code(self, symbols, indexes):
        """RansEncoder.encode_with_indexes over one image's flattened symbols"""
        from .coder import RansEncoder

        cdf, sizes, offsets = self.host_tables()
        return RansEncoder().encode_with_indexes(symbols, indexes, cdf, sizes, offsets)

    def _decode(self, string, indexes):
        from .coder import RansDecoder

        cdf, sizes, offsets = self.host_tables()
        dec = RansDecoder()
        dec.set_stream(string)
        return dec.decode_stream_array(indexes, cdf, sizes, offsets)


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

    def loss(self):
        """aux loss sum |f(quantiles) - target| (utils/engine.py:79); differentiable w.r.t. quantiles"""
        if torch.is_grad_enabled() and self.quantiles.requires_grad:
            from .mcm_train import AuxLossFn

            return AuxLossFn.apply(self, self.quantiles)
        with torch.no_grad():
            return ops.eb_aux_loss(self)

    @torch.no_grad()
    def update(self, force=False):
        """EntropyBottleneck.update: per-channel integer support around the median, pmf of every
        integer (device kernel), quantized CDF with the tail mass as the escape bin."""
        if self._offset.numel() > 0 and not force:
            return False
        medians = self.quantiles[:, 0, 1]
        minima = torch.clamp(torch.ceil(medians - self.quantiles[:, 0, 0]).int(), min=0)
        maxima = torch.clamp(torch.ceil(self.quantiles[:, 0, 2] - medians).int(), min=0)
        self._offset = -minima
        pmf_start = medians - minima
        pmf_length = maxima + minima + 1
        max_length = int(pmf_length.max().item())
        pmf, tail = ops.eb_pmf(self, pmf_start, max_length)
        self._quantized_cdf = self._pmf_to_cdf(pmf, tail, pmf_length, max_length)
        self._cdf_length = pmf_length + 2
        return True

    def _channel_indexes(self, hw):
        return np.repeat(np.arange(self.channels, dtype=np.int32), hw)

    @torch.no_grad()
    def compress(self, x):
        """x NCHW -> one rANS string per image (symbols round(x - median), channel-indexed CDFs)"""
        n, c, h, w = x.shape
        z = x.float().permute(0, 2, 3, 1).contiguous()
        sym = ops.eb_symbols(self, z, n, c, h * w).cpu().numpy()
        idx = self._channel_indexes(h * w)
        return [self._code(sym[i].reshape(-1), idx) for i in range(n)]

    @torch.no_grad()
    def decompress(self, strings, size):
        """strings -> z_hat NCHW f32 (symbols + median)"""
        h, w = int(size[0]), int(size[1])
        n, c = len(strings), self.channels
        idx = self._channel_indexes(h * w)
        sym = np.stack([self._decode(s, idx) for s in strings]).astype(np.int32)
        dev = self.quantiles.device
        zhat = torch.empty((n * h * w, c), dtype=torch.float32, device=dev)
        ops.eb_dequantize(self, torch.from_numpy(sym).to(dev), n, c, h * w, zhat)
        return zhat.view(n, h, w, c).permute(0, 3, 1, 2).contiguous()


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

    @staticmethod
    def _prepare_scale_table(scale_table):
        return torch.Tensor(tuple(float(s) for s in scale_table))

    @staticmethod
    def _standardized_quantile(quantile):
        from scipy.stats import norm

        return float(norm.ppf(quantile))

    @torch.no_grad()
    def update_scale_table(self, scale_table, force=False):
        if self._offset.numel() > 0 and not force:
            return False
        device = self.scale_table.device
        self.scale_table = self._prepare_scale_table(scale_table).to(device)
        self.update()
        return True

    @torch.no_grad()
    def update(self):
        """GaussianConditional.update: one discretised-Gaussian CDF per scale-table entry, support
        +-ceil(scale * Phi^-1(1 - tail_mass / 2)) (pmf on the device, CDF builder on the host)."""
        multiplier = -self._standardized_quantile(self.tail_mass / 2)
        pmf_center = torch.ceil(self.scale_table * multiplier).int()
        pmf_length = 2 * pmf_center + 1
        max_length = int(torch.max(pmf_length).item())
        pmf, tail = ops.gc_pmf(self.scale_table.float(), pmf_center, max_length)
        self._quantized_cdf = self._pmf_to_cdf(pmf, tail, pmf_length, max_length)
        self._offset = -pmf_center
        self._cdf_length = pmf_length + 2

    def build_indexes(self, scales):
        """index of the smallest table scale >= max(scales, bound) (module-level convenience; MCM.compress
        computes indexes inside the fused slice kernel)"""
        scales = self.lower_bound_scale(scales)
        indexes = scales.new_full(scales.size(), len(self.scale_table) - 1).int()
        for s in self.scale_table[:-1]:
            indexes -= (scales <= s).int()
        return indexes

    @torch.no_grad()
    def compress(self, inputs, indexes, means=None):
        sym = self.quantize_symbols(inputs, means).cpu().numpy().reshape(inputs.shape[0], -1)
        idx = indexes.int().cpu().numpy().reshape(inputs.shape[0], -1)
        return [self._code(sym[i], idx[i]) for i in range(sym.shape[0])]

    @torch.no_grad()
    def decompress(self, strings, indexes, dtype=torch.float, means=None):
        idx = indexes.int().cpu().numpy().reshape(len(strings), -1)
        out = torch.from_numpy(np.stack([self._decode(s, idx[i]) for i, s in enumerate(strings)]))
        out = out.reshape(indexes.shape).to(indexes.device)
        return self.dequantize(out, means, dtype)


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

    def update(self, scale_table=None, force=False):
        """CompressionModel.update (testing.py:223): build the CDF tables of every entropy model"""
        if scale_table is None:
            scale_table = get_scale_table()
        updated = False
        for _, module in self.named_modules():
            if isinstance(module, EntropyBottleneck):
                updated |= module.update(force=force)
            if isinstance(module, GaussianConditional):
                updated |= module.update_scale_table(scale_table, force=force)
        return updated

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
