"""ORACLE — test infrastructure only.

Functional CPU restatement of the reference hot path, ``MCM.forward`` (reference
models/Compression/MCM.py:714-803) and its helpers, on plain tensors taken from a state_dict
with the reference's key names.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it; the product path never imports anything under ``oracle/``.

Third-party arithmetic (timm Block / PatchEmbed, compressai entropy models) is restated in
``oracle/thirdparty.py``; the glue here is pinned by the golden fixtures that
``tools/gen_golden.py`` produced by running the REAL reference glue (see tests/test_oracle.py).

Runs in float32 by default; pass ``dtype=torch.float64`` for a high-precision reference.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from . import ids as ids_oracle


@dataclass
class MCMConfig:
    """MCM constructor arguments (MCM.py:34-52) — same names and defaults."""
    img_size: int = 224
    patch_size: int = 16
    in_chans: int = 3
    encoder_embed_dim: int = 768
    encoder_depth: int = 12
    encoder_num_heads: int = 12
    decoder_embed_dim: int = 512
    decoder_depth: int = 8
    decoder_num_heads: int = 16
    mlp_ratio: float = 4.0
    norm_eps: float = 1e-6
    latent_depth: int = 384
    hyperprior_depth: int = 192
    num_slices: int = 12
    num_keep_patches: int = 144

    def kwargs(self):
        d = dict(self.__dict__)
        d.pop("norm_eps")
        return d


# ------------------------------------------------------------------------------ building blocks
def layer_norm(x, sd, pre, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[pre + "weight"], sd[pre + "bias"], eps)


def linear(x, sd, pre):
    return F.linear(x, sd[pre + "weight"], sd.get(pre + "bias"))


def block(x, sd, pre, heads, eps):
    """timm 0.4.5 Block (pre-LN, qkv_bias=True, exact-erf GELU)."""
    b, n, c = x.shape
    h = layer_norm(x, sd, pre + "norm1.", eps)
    qkv = linear(h, sd, pre + "attn.qkv.").reshape(b, n, 3, heads, c // heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    attn = ((q @ k.transpose(-2, -1)) * ((c // heads) ** -0.5)).softmax(dim=-1)
    a = (attn @ v).transpose(1, 2).reshape(b, n, c)
    x = x + linear(a, sd, pre + "attn.proj.")
    h = layer_norm(x, sd, pre + "norm2.", eps)
    return x + linear(F.gelu(linear(h, sd, pre + "mlp.fc1.")), sd, pre + "mlp.fc2.")


def conv(x, sd, pre, stride=1, padding=1):
    return F.conv2d(x, sd[pre + "weight"], sd[pre + "bias"], stride=stride, padding=padding)


def seq_convs(x, sd, pre, layers):
    """nn.Sequential of convs with GELU in between; `layers` = list of (index, kind, stride)."""
    for j, (idx, kind, stride) in enumerate(layers):
        if kind == "conv":
            x = conv(x, sd, f"{pre}{idx}.", stride)
        elif kind == "subpel":  # compressai subpel_conv3x3(r=2): conv -> PixelShuffle(2)
            x = F.pixel_shuffle(conv(x, sd, f"{pre}{idx}.0."), 2)
        elif kind == "conv1x1":
            x = conv(x, sd, f"{pre}{idx}.", 1, 0)
        elif kind == "convT1x1":
            x = F.conv_transpose2d(x, sd[f"{pre}{idx}.weight"], sd[f"{pre}{idx}.bias"])
        if j < len(layers) - 1:
            x = F.gelu(x)
    return x


G_A = [(0, "conv1x1", 1), (2, "conv1x1", 1), (4, "conv1x1", 1), (6, "conv1x1", 1)]
G_S = [(0, "convT1x1", 1), (2, "convT1x1", 1), (4, "convT1x1", 1), (6, "convT1x1", 1)]
H_A = [(0, "conv", 1), (2, "conv", 1), (4, "conv", 2), (6, "conv", 1), (8, "conv", 2)]
H_S = [(0, "conv", 1), (2, "subpel", 1), (4, "conv", 1), (6, "subpel", 1), (8, "conv", 1)]
CC = [(0, "conv", 1), (2, "conv", 1), (4, "conv", 1), (6, "conv", 1), (8, "conv", 1)]


def eb_logits(sd, pre, x):
    """compressai EntropyBottleneck._logits_cumulative, x: [C, 1, n]"""
    logits = x
    for i in range(5):
        logits = torch.matmul(F.softplus(sd[f"{pre}_matrix{i}"]), logits) + sd[f"{pre}_bias{i}"]
        if i < 4:
            logits = logits + torch.tanh(sd[f"{pre}_factor{i}"]) * torch.tanh(logits)
    return logits


def entropy_bottleneck(sd, pre, z, noise=None):
    """EntropyBottleneck.forward: returns (likelihood NCHW, z_hat = round(z - med) + med)."""
    c = z.shape[1]
    values = z.permute(1, 0, 2, 3).reshape(c, 1, -1)
    med = sd[pre + "quantiles"][:, :, 1:2]
    if noise is not None:
        x = values + noise.permute(1, 0, 2, 3).reshape(c, 1, -1).to(z.dtype)
    else:
        x = torch.round(values - med) + med
    lower = eb_logits(sd, pre, x - 0.5)
    upper = eb_logits(sd, pre, x + 0.5)
    sign = -torch.sign(lower + upper)
    lik = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))
    lik = torch.clamp_min(lik, 1e-9)
    lik = lik.reshape(c, z.shape[0], z.shape[2], z.shape[3]).permute(1, 0, 2, 3).contiguous()
    med4 = med.reshape(1, c, 1, 1)
    z_hat = torch.round(z - med4) + med4
    return lik, z_hat


def eb_aux_loss(sd, pre):
    logits = eb_logits(sd, pre, sd[pre + "quantiles"])
    return torch.abs(logits - sd[pre + "target"].to(logits.dtype)).sum()


def gaussian_conditional(y, sigma, mu, noise=None, scale_bound=0.11):
    yt = y + noise.to(y.dtype) if noise is not None else torch.round(y - mu) + mu
    values = torch.abs(yt - mu)
    s = torch.clamp_min(sigma, scale_bound)
    c = float(-(2 ** -0.5))
    upper = 0.5 * torch.erfc(c * ((0.5 - values) / s))
    lower = 0.5 * torch.erfc(c * ((-0.5 - values) / s))
    return torch.clamp_min(upper - lower, 1e-9)


def unpatchify(x, p, c=3):
    n, l, _ = x.shape
    h = w = int(round(l ** 0.5))
    x = x.reshape(n, h, w, p, p, c)
    x = torch.einsum("nhwpqc->nchpwq", x)
    return x.reshape(n, c, h * p, w * p)


def patchify(imgs, p):
    n, c, hh, ww = imgs.shape
    h = w = hh // p
    x = imgs.reshape(n, c, h, p, w, p)
    x = torch.einsum("nchpwq->nhwpqc", x)
    return x.reshape(n, h * w, p * p * c)


# ------------------------------------------------------------------------------ MCM.forward
@dataclass
class OracleOut:
    x_hat: torch.Tensor
    y_likelihood: torch.Tensor
    z_likelihood: torch.Tensor
    ids_shuffle: torch.Tensor
    ids_restore: torch.Tensor
    inter: dict = field(default_factory=dict)


def mcm_forward(sd, cfg: MCMConfig, imgs, scores, z_noise=None, y_noise=None, lanes=8, dtype=torch.float32,
                keep_intermediates=False) -> OracleOut:
    """MCM.forward (MCM.py:714-803) without forward_loss.  Training mode <=> noise given."""
    sd = {k: (v.to(dtype) if torch.is_floating_point(v) else v) for k, v in sd.items()}
    imgs = imgs.to(dtype)
    inter = {}
    p, K, D = cfg.patch_size, cfg.num_keep_patches, cfg.encoder_embed_dim
    n = imgs.shape[0]

    # --- forward_encoder (MCM.py:590-634)
    shuf, rest = ids_oracle.ids_shuffle(scores.float().cpu().numpy(), K, lanes)
    shuf = torch.from_numpy(shuf)
    rest = torch.from_numpy(rest)
    x = F.conv2d(imgs, sd["encoder_embed.proj.weight"], sd["encoder_embed.proj.bias"], stride=p)
    x = x.flatten(2).transpose(1, 2)
    pos = sd["encoder_pos_embed"]
    x = x + pos[:, 1:, :]
    x = torch.gather(x, 1, shuf[:, :K].unsqueeze(-1).repeat(1, 1, D))
    cls = (sd["cls_token"] + pos[:, :1, :]).expand(n, -1, -1)
    x = torch.cat((cls, x), dim=1)
    for i in range(cfg.encoder_depth):
        x = block(x, sd, f"encoder_blocks.{i}.", cfg.encoder_num_heads, cfg.norm_eps)
    x = layer_norm(x, sd, "encoder_norm.", cfg.norm_eps)[:, 1:, :]
    if keep_intermediates:
        inter["enc_out"] = x

    # --- LIC (MCM.py:729-787)
    g = int(K ** 0.5)
    y = x.reshape(-1, g, g, D).permute(0, 3, 1, 2).contiguous()
    y = seq_convs(y, sd, "g_a.", G_A)
    z = seq_convs(y, sd, "h_a.", H_A)
    z_lik, z_hat = entropy_bottleneck(sd, "entropy_bottleneck.", z, z_noise)
    ls = seq_convs(z_hat, sd, "h_s_scale.", H_S)
    lm = seq_convs(z_hat, sd, "h_s_mean.", H_S)
    if keep_intermediates:
        inter.update(y=y, z=z, z_hat=z_hat, latent_scales=ls, latent_means=lm)
    S = cfg.num_slices
    maxsup = S // 2
    hh, ww = y.shape[2:]
    y_slices = y.chunk(S, 1)
    y_noise_slices = y_noise.to(dtype).chunk(S, 1) if y_noise is not None else [None] * S
    yhat, liks = [], []
    for i, ys in enumerate(y_slices):
        sup = yhat[:maxsup]
        mean_support = torch.cat([lm] + sup, dim=1)
        mu = seq_convs(mean_support, sd, f"cc_transform_mean.{i}.", CC)[:, :, :hh, :ww]
        scale_support = torch.cat([ls] + sup, dim=1)
        sigma = seq_convs(scale_support, sd, f"cc_transform_scale.{i}.", CC)[:, :, :hh, :ww]
        liks.append(gaussian_conditional(ys, sigma, mu, y_noise_slices[i]))
        yh = torch.round(ys - mu) + mu
        lrp = seq_convs(torch.cat([mean_support, yh], dim=1), sd, f"lrp_transform.{i}.", CC)
        yh = yh + 0.5 * torch.tanh(lrp)
        yhat.append(yh)
        if keep_intermediates:
            inter[f"mu{i}"], inter[f"sigma{i}"] = mu, sigma
    y_hat = torch.cat(yhat, dim=1)
    y_lik = torch.cat(liks, dim=1)
    if keep_intermediates:
        inter["y_hat"] = y_hat
    t = seq_convs(y_hat, sd, "g_s.", G_S)
    t = t.permute(0, 2, 3, 1).contiguous().view(-1, K, D)

    # --- forward_decoder (MCM.py:636-688), including the off-by-one "cls" of the reference
    xd = linear(t, sd, "decoder_embed.")
    L = rest.shape[1]
    mask = sd["mask_token"].repeat(n, L + 1 - xd.shape[1], 1)
    x_ = torch.cat([xd[:, 1:, :], mask], dim=1)
    x_ = torch.gather(x_, 1, rest.unsqueeze(-1).repeat(1, 1, xd.shape[2]))
    x = torch.cat([xd[:, :1, :], x_], dim=1) + sd["decoder_pos_embed"]
    for i in range(cfg.decoder_depth):
        x = block(x, sd, f"decoder_blocks.{i}.", cfg.decoder_num_heads, cfg.norm_eps)
    x = layer_norm(x, sd, "decoder_norm.", cfg.norm_eps)
    preds = linear(x, sd, "decoder_pred.")[:, 1:, :]
    x_hat = unpatchify(preds, p, cfg.in_chans)
    return OracleOut(x_hat, y_lik, z_lik, shuf, rest, inter)


def forward_loss(x_hat, imgs):
    """MCM.forward_loss (MCM.py:690-712) without the VGG term (weights need a download)."""
    from .thirdparty import ssim

    return 1 - ssim(x_hat, imgs, data_range=1), F.l1_loss(x_hat, imgs)


def rate_bpp(y_lik, z_lik, num_pixels):
    """RateDistortionLoss bpp term (models/Compression/loss/rd_loss.py:19-20)."""
    return sum(torch.log(l).sum() / (-math.log(2) * num_pixels) for l in (y_lik, z_lik))


# ------------------------------------------------------------------------------ parameters
def pos_embed_2d(embed_dim, grid_size, cls_token=True):
    """get_2d_sincos_pos_embed (models/Compression/common/pos_embed.py:23-94), float64 numpy."""
    gh = np.arange(grid_size, dtype=np.float32)
    gw = np.arange(grid_size, dtype=np.float32)
    grid = np.stack(np.meshgrid(gw, gh), axis=0).reshape(2, 1, grid_size, grid_size)

    def one_d(d, pos):
        omega = np.arange(d // 2, dtype=np.float64) / (d / 2.0)
        omega = 1.0 / 10000 ** omega
        out = np.einsum("m,d->md", pos.reshape(-1), omega)
        return np.concatenate([np.sin(out), np.cos(out)], axis=1)

    emb = np.concatenate([one_d(embed_dim // 2, grid[0]), one_d(embed_dim // 2, grid[1])], axis=1)
    if cls_token:
        emb = np.concatenate([np.zeros([1, embed_dim]), emb], axis=0)
    return emb


def _shapes(cfg: MCMConfig):
    """state_dict (name -> shape) of the reference MCM for `cfg` (MCM.py:71-354)."""
    E, Dd, M, N, S = cfg.encoder_embed_dim, cfg.decoder_embed_dim, cfg.latent_depth, cfg.hyperprior_depth, cfg.num_slices
    P, C = cfg.patch_size, cfg.in_chans
    L = (cfg.img_size // P) ** 2
    sh = {}
    eb = "entropy_bottleneck."
    filt = (1, 3, 3, 3, 3, 1)
    for i in range(5):
        sh[f"{eb}_matrix{i}"] = (N, filt[i + 1], filt[i])
        sh[f"{eb}_bias{i}"] = (N, filt[i + 1], 1)
        if i < 4:
            sh[f"{eb}_factor{i}"] = (N, filt[i + 1], 1)
    sh[eb + "quantiles"] = (N, 1, 3)
    ga = [E, int(Dd + (E - Dd) * 3 / 4), int(Dd + (E - Dd) * 2 / 4), Dd, M]
    for j in range(4):
        sh[f"g_a.{2 * j}.weight"] = (ga[j + 1], ga[j], 1, 1)
        sh[f"g_a.{2 * j}.bias"] = (ga[j + 1],)
    gs = ga[::-1]
    for j in range(4):
        sh[f"g_s.{2 * j}.weight"] = (gs[j], gs[j + 1], 1, 1)  # ConvTranspose2d: [in, out, 1, 1]
        sh[f"g_s.{2 * j}.bias"] = (gs[j + 1],)
    ha = [M, M, int(N + (M - N) * 3 / 4), int(N + (M - N) * 2 / 4), int(N + (M - N) / 4), N]
    for j in range(5):
        sh[f"h_a.{2 * j}.weight"] = (ha[j + 1], ha[j], 3, 3)
        sh[f"h_a.{2 * j}.bias"] = (ha[j + 1],)
    hs = [N, int(N + (M - N) / 4), int(N + (M - N) * 2 / 4), int(N + (M - N) * 3 / 4), M, M]
    for name in ("h_s_mean", "h_s_scale"):
        for j in range(5):
            cout = hs[j + 1] * (4 if j in (1, 3) else 1)
            key = f"{name}.{2 * j}.0." if j in (1, 3) else f"{name}.{2 * j}."
            sh[key + "weight"] = (cout, hs[j], 3, 3)
            sh[key + "bias"] = (cout,)
    sw = M // S
    mid = [int(sw * (S // 2 + 1)), int(sw * (S // 2 * 3 / 4 + 1)), int(sw * (S // 2 * 2 / 4 + 1)),
           int(sw * (S // 2 * 1 / 4 + 1)), sw]
    for name in ("cc_transform_mean", "cc_transform_scale", "lrp_transform"):
        for i in range(S):
            cin = int(M + sw * min(i, S // 2)) if name != "lrp_transform" else int(M + sw * min(i + 1, S // 2 + 1))
            chans = [cin] + mid
            for j in range(5):
                sh[f"{name}.{i}.{2 * j}.weight"] = (chans[j + 1], chans[j], 3, 3)
                sh[f"{name}.{i}.{2 * j}.bias"] = (chans[j + 1],)
    sh["cls_token"] = (1, 1, E)
    sh["encoder_pos_embed"] = (1, L + 1, E)
    sh["encoder_embed.proj.weight"] = (E, C, P, P)
    sh["encoder_embed.proj.bias"] = (E,)

    def blk(pre, d, r):
        h = int(d * r)
        return {pre + "norm1.weight": (d,), pre + "norm1.bias": (d,), pre + "attn.qkv.weight": (3 * d, d),
                pre + "attn.qkv.bias": (3 * d,), pre + "attn.proj.weight": (d, d), pre + "attn.proj.bias": (d,),
                pre + "norm2.weight": (d,), pre + "norm2.bias": (d,), pre + "mlp.fc1.weight": (h, d),
                pre + "mlp.fc1.bias": (h,), pre + "mlp.fc2.weight": (d, h), pre + "mlp.fc2.bias": (d,)}

    for i in range(cfg.encoder_depth):
        sh.update(blk(f"encoder_blocks.{i}.", E, cfg.mlp_ratio))
    sh["encoder_norm.weight"] = (E,)
    sh["encoder_norm.bias"] = (E,)
    sh["decoder_embed.weight"] = (Dd, E)
    sh["decoder_embed.bias"] = (Dd,)
    sh["mask_token"] = (1, 1, Dd)
    sh["decoder_pos_embed"] = (1, L + 1, Dd)
    for i in range(cfg.decoder_depth):
        sh.update(blk(f"decoder_blocks.{i}.", Dd, cfg.mlp_ratio))
    sh["decoder_norm.weight"] = (Dd,)
    sh["decoder_norm.bias"] = (Dd,)
    sh["decoder_pred.weight"] = (P * P * C, Dd)
    sh["decoder_pred.bias"] = (P * P * C,)
    return sh


def make_state_dict(cfg: MCMConfig, seed: int = 0):
    """Deterministic, platform-independent weights (numpy PCG64), fan-in scaled so activations stay
    O(1) through the whole stack; LayerNorm / entropy-model parameters randomised around their
    defaults so every code path (GELU, tanh factors, noise) is exercised."""
    rng = np.random.default_rng(seed)
    sd = {}
    for k, shp in _shapes(cfg).items():
        if k.endswith("pos_embed"):
            g = int(round((shp[1] - 1) ** 0.5))
            sd[k] = torch.from_numpy(pos_embed_2d(shp[2], g)).float().unsqueeze(0)
            continue
        if "entropy_bottleneck" in k:
            if "quantiles" in k:
                v = np.array([-10.0, 0.0, 10.0])[None, None, :] + rng.uniform(-0.3, 0.3, shp)
            elif "_matrix" in k:
                v = rng.normal(0.0, 0.5, shp)
            elif "_factor" in k:
                v = rng.normal(0.0, 0.5, shp)
            else:
                v = rng.uniform(-0.5, 0.5, shp)
        elif k.endswith("norm1.weight") or k.endswith("norm2.weight") or k.endswith("norm.weight"):
            v = 1.0 + 0.1 * rng.standard_normal(shp)
        elif k.endswith(".bias") or k.endswith("bias"):
            v = 0.02 * rng.standard_normal(shp)
        elif k in ("cls_token", "mask_token"):
            v = 0.02 * rng.standard_normal(shp)
        else:
            if len(shp) == 4 and k.startswith("g_s."):
                fan_in = shp[0]
            else:
                fan_in = int(np.prod(shp[1:]))
            v = rng.standard_normal(shp) / math.sqrt(fan_in)
        sd[k] = torch.from_numpy(np.asarray(v, dtype=np.float32))
    sd["entropy_bottleneck.target"] = torch.Tensor([-np.log(2 / 1e-9 - 1), 0, np.log(2 / 1e-9 - 1)])
    return sd
