"""TEST INFRASTRUCTURE ONLY -- CPU restatement (torch f32) of compressai 1.2.4's CDF-table updates
and of MCM.compress's symbol / index streams, the checker for the device coding kernels.
Imported only by tests/.

References: EntropyBottleneck.update / GaussianConditional.update(_scale_table) / build_indexes
(compressai, called via CompressionModel.update at testing.py:223) and MCM.compress
(models/Compression/MCM.py:805-894: z strings per image from EntropyBottleneck.compress, ONE y string
with symbols = round(y - mu) and indexes = build_indexes(sigma), slice-major, each slice [N,32,H,W]).
compressai is not vendored/installed: **parity unpinned** against the package itself.
"""
from __future__ import annotations

import torch
from scipy.stats import norm

from . import rans_oracle as ro
from .mcm_oracle import eb_logits


def _tables(pmf, tail, lengths, max_length, precision=16):
    """EntropyModel._pmf_to_cdf"""
    cdf = torch.zeros((len(lengths), max_length + 2), dtype=torch.int32)
    for i, n in enumerate(lengths):
        prob = torch.cat([pmf[i, :n], tail[i:i + 1]]).numpy()
        row = ro.pmf_to_quantized_cdf(prob, precision)
        cdf[i, :len(row)] = torch.tensor(row, dtype=torch.int32)
    return cdf


def eb_update(sd, pre="entropy_bottleneck."):
    """-> (quantized_cdf [C][max+2], cdf_length [C], offset [C])"""
    q = sd[pre + "quantiles"].float()
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = int(pmf_length.max())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    lower = eb_logits(sd, pre, samples - 0.5)
    upper = eb_logits(sd, pre, samples + 0.5)
    sign = -torch.sign(lower + upper)
    pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
    tail = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    return _tables(pmf, tail[:, 0], pmf_length.tolist(), max_length), pmf_length + 2, -minima


def eb_pmf(sd, pre="entropy_bottleneck."):
    q = sd[pre + "quantiles"].float()
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    max_length = int((maxima + minima + 1).max())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    lower = eb_logits(sd, pre, samples - 0.5)
    upper = eb_logits(sd, pre, samples + 0.5)
    sign = -torch.sign(lower + upper)
    pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
    return pmf, (torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:]))[:, 0], pmf_start, max_length


def gc_pmf(scale_table, tail_mass=1e-9):
    table = scale_table.float()
    pmf_center = torch.ceil(table * -float(norm.ppf(tail_mass / 2))).int()
    max_length = int((2 * pmf_center + 1).max())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    sc = table.unsqueeze(1)
    c = float(-(2 ** -0.5))
    upper = 0.5 * torch.erfc(c * ((0.5 - samples) / sc))
    lower = 0.5 * torch.erfc(c * ((-0.5 - samples) / sc))
    return upper - lower, 2 * lower[:, 0], pmf_center, max_length


def gc_update(scale_table, tail_mass=1e-9):
    table = scale_table.float()
    multiplier = -float(norm.ppf(tail_mass / 2))
    pmf_center = torch.ceil(table * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = int(pmf_length.max())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    sc = table.unsqueeze(1)
    c = float(-(2 ** -0.5))
    upper = 0.5 * torch.erfc(c * ((0.5 - samples) / sc))
    lower = 0.5 * torch.erfc(c * ((-0.5 - samples) / sc))
    pmf = upper - lower
    tail = 2 * lower[:, 0]
    return _tables(pmf, tail, pmf_length.tolist(), max_length), pmf_length + 2, -pmf_center


def build_indexes(sigma, scale_table, bound=0.11):
    s = torch.clamp_min(sigma, bound)
    idx = torch.full(s.shape, len(scale_table) - 1, dtype=torch.int32)
    for t in scale_table[:-1]:
        idx -= (s <= t).int()
    return idx


def compress_streams(inter, num_slices, scale_table, sd, pre="entropy_bottleneck."):
    """symbol / index arrays MCM.compress hands to the coder, from mcm_forward(keep_intermediates=True)"""
    y, z = inter["y"], inter["z"]
    med = sd[pre + "quantiles"][:, 0, 1].reshape(1, -1, 1, 1)
    zsym = torch.round(z - med).int().reshape(z.shape[0], -1)
    ysym, yidx = [], []
    for i, ys in enumerate(y.chunk(num_slices, 1)):
        mu, sigma = inter[f"mu{i}"], inter[f"sigma{i}"]
        ysym.append(torch.round(ys - mu).int().reshape(-1))
        yidx.append(build_indexes(sigma, scale_table).reshape(-1))
    return zsym, torch.cat(ysym), torch.cat(yidx)
