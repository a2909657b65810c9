"""ORACLE — test infrastructure only (checker for the training path's gradients).

Autograd-faithful functional restatement of the reference training forward, ``MCM.forward`` in
``model.train()`` (models/Compression/MCM.py:714-803), for torch.autograd on the CPU:

  * compressai 1.2.4 ``LowerBound`` backward (LowerBoundFunction: the gradient passes where
    x >= bound or grad < 0) for the likelihood bound 1e-9 and the scale bound 0.11;
  * ``quantize_ste`` (round(x) - x).detach() + x for z_hat (MCM.py:742-744) and y_hat (MCM.py:776);
  * training-mode entropy models: likelihood of x + U(-1/2, 1/2) with injected noise;
  * EntropyBottleneck._likelihood's detached sign; aux loss with stop_gradient (engine.py:79).

Everything else (blocks, convs, glue, the decoder's off-by-one cls) is mcm_oracle's restatement,
which tests/test_oracle.py pins against the reference's own outputs.  The gradients themselves are
"parity unpinned" against compressai / timm (absent here); they follow the published semantics.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import ids as ids_oracle
from .mcm_oracle import CC, G_A, G_S, H_A, H_S, MCMConfig, block, eb_logits, layer_norm, linear, seq_convs, unpatchify


class LowerBoundFn(torch.autograd.Function):
    """compressai.ops.bound_ops.LowerBoundFunction"""

    @staticmethod
    def forward(ctx, x, bound):
        b = torch.tensor(float(bound), dtype=x.dtype)
        ctx.save_for_backward(x, b)
        return torch.max(x, b)

    @staticmethod
    def backward(ctx, g):
        x, b = ctx.saved_tensors
        pass_through = (x >= b) | (g < 0)
        return pass_through.to(g.dtype) * g, None


def lower_bound(x, bound):
    return LowerBoundFn.apply(x, bound)


def quantize_ste(x):
    return (torch.round(x) - x).detach() + x


def eb_train(sd, pre, z, noise):
    """EntropyBottleneck.forward (training) -> (likelihood NCHW, z_hat = quantize_ste(z - med) + med)"""
    n, c, h, w = z.shape
    values = z.permute(1, 0, 2, 3).reshape(c, 1, -1)
    x = values + noise.to(z.dtype).permute(1, 0, 2, 3).reshape(c, 1, -1)
    lower = eb_logits(sd, pre, x - 0.5)
    upper = eb_logits(sd, pre, x + 0.5)
    sign = (-torch.sign(lower + upper)).detach()
    lik = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))
    lik = lower_bound(lik, 1e-9)
    lik = lik.reshape(c, n, h, w).permute(1, 0, 2, 3)
    med = sd[pre + "quantiles"][:, :, 1:2].reshape(1, c, 1, 1)
    z_hat = quantize_ste(z - med) + med
    return lik, z_hat


def gc_train(y, sigma, mu, noise):
    """GaussianConditional.forward (training): likelihood of y + noise"""
    values = torch.abs((y + noise.to(y.dtype)) - mu)
    s = lower_bound(sigma, 0.11)
    c = float(-(2 ** -0.5))
    upper = 0.5 * torch.erfc(c * ((0.5 - values) / s))
    lower = 0.5 * torch.erfc(c * ((-0.5 - values) / s))
    return lower_bound(upper - lower, 1e-9)


def aux_loss(sd, pre):
    """EntropyBottleneck.loss: stop_gradient on the density parameters, gradient to quantiles only"""
    det = {k: (v.detach() if k.startswith(pre) and not k.endswith("quantiles") else v) for k, v in sd.items()}
    logits = eb_logits(det, pre, sd[pre + "quantiles"])
    return torch.abs(logits - sd[pre + "target"].to(logits.dtype)).sum()


def mcm_forward_train(sd, cfg: MCMConfig, imgs, scores, z_noise, y_noise, lanes=8):
    """MCM.forward (training mode) without forward_loss -> (x_hat, y_likelihood, z_likelihood)"""
    p, K, D = cfg.patch_size, cfg.num_keep_patches, cfg.encoder_embed_dim
    n = imgs.shape[0]
    shuf, rest = ids_oracle.ids_shuffle(scores.float().cpu().numpy(), K, lanes)
    shuf, rest = torch.from_numpy(shuf), torch.from_numpy(rest)
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

    g = int(K ** 0.5)
    y = x.reshape(-1, g, g, D).permute(0, 3, 1, 2).contiguous()
    y = seq_convs(y, sd, "g_a.", G_A)
    z = seq_convs(y, sd, "h_a.", H_A)
    z_lik, z_hat = eb_train(sd, "entropy_bottleneck.", z, z_noise)
    ls = seq_convs(z_hat, sd, "h_s_scale.", H_S)
    lm = seq_convs(z_hat, sd, "h_s_mean.", H_S)
    S = cfg.num_slices
    maxsup = S // 2
    hh, ww = y.shape[2:]
    yn = y_noise.to(y.dtype).chunk(S, 1)
    yhat, liks = [], []
    for i, ys in enumerate(y.chunk(S, 1)):
        sup = yhat[:maxsup]
        mean_support = torch.cat([lm] + sup, dim=1)
        mu = seq_convs(mean_support, sd, f"cc_transform_mean.{i}.", CC)[:, :, :hh, :ww]
        scale_support = torch.cat([ls] + sup, dim=1)
        sigma = seq_convs(scale_support, sd, f"cc_transform_scale.{i}.", CC)[:, :, :hh, :ww]
        liks.append(gc_train(ys, sigma, mu, yn[i]))
        yh = quantize_ste(ys - mu) + mu
        lrp = seq_convs(torch.cat([mean_support, yh], dim=1), sd, f"lrp_transform.{i}.", CC)
        yhat.append(yh + 0.5 * torch.tanh(lrp))
    y_hat = torch.cat(yhat, dim=1)
    y_lik = torch.cat(liks, dim=1)
    t = seq_convs(y_hat, sd, "g_s.", G_S)
    t = t.permute(0, 2, 3, 1).contiguous().view(-1, K, D)

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
    return unpatchify(preds, p, cfg.in_chans), y_lik, z_lik


def rate_bpp(y_lik, z_lik, num_pixels):
    """RateDistortionLoss bpp term (rd_loss.py:19-20)"""
    return sum(torch.log(lik).sum() / (-math.log(2) * num_pixels) for lik in (y_lik, z_lik))
