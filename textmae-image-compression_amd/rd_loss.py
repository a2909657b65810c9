"""RateDistortionLoss — counterpart of reference models/Compression/loss/rd_loss.py:7-28.

Same constructor (`lmbda`), same output keys ("bpp_loss", "ssim_loss", "L1_loss", "vgg_loss", "loss")
and the same formula: loss = lmbda * (0.25*ssim + 10*L1 + 0.1*vgg) + bpp.  The bpp reduction over
both likelihood tensors runs on the device (tmae_bpp_sum).
"""
import torch
import torch.nn as nn

from . import ops


class RateDistortionLoss(nn.Module):
    def __init__(self, lmbda=1e-2):
        super().__init__()
        self.lmbda = lmbda

    def forward(self, output, target):
        N, _, H, W = target.size()
        out = {}
        lik = output["likelihoods"]
        if torch.is_grad_enabled() and (lik["y"].requires_grad or lik["z"].requires_grad):
            from .mcm_train import BppFn

            out["bpp_loss"] = BppFn.apply(lik["y"], lik["z"], N * H * W)
        else:
            out["bpp_loss"] = ops.bpp(lik["y"], lik["z"], N * H * W)
        out["ssim_loss"] = output["loss"][0]
        out["L1_loss"] = output["loss"][1]
        out["vgg_loss"] = output["loss"][2]
        out["loss"] = self.lmbda * (0.25 * out["ssim_loss"] + 10 * out["L1_loss"] + 0.1 * out["vgg_loss"]) \
            + out["bpp_loss"]
        return out
