"""Why does optim.clip_grad_norm_ fall back to torch's foreach path in the training step?  Prints, after one
engine.train_step's main backward, which parameters' gradients are not views of the executor's flat buffer."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import textmae_amd  # noqa: E402
from textmae_amd.optim import _flat_owner, configure_optimizers  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402

torch.manual_seed(0)
m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
m.compute_dtype = torch.bfloat16
m.distortion = "ssim+l1"
opt, aux = configure_optimizers(m, fused=True)
crit = RateDistortionLoss(lmbda=1e-2)
x = torch.rand(4, 3, 256, 256, device="cuda")
s = torch.rand(4, 256, device="cuda")
for step in range(2):
    out = m(x, s)
    loss = crit(out, x)["loss"]
    loss.backward()
    params = [p for p in m.parameters() if p.grad is not None]
    gs = [p.grad for p in params]
    base = gs[0]._base
    names = {id(p): n for n, p in m.named_parameters()}
    bad = [names[id(p)] for p in params if p.grad._base is None or p.grad._base is not base]
    nograd = [n for n, p in m.named_parameters() if p.requires_grad and p.grad is None]
    print(f"step {step}: {len(params)} grads, base numel {None if base is None else base.numel()}, "
          f"sum {sum(g.numel() for g in gs)}, not views of base: {bad[:10]} ({len(bad)}), no grad: {nograd[:10]}")
    print("flat owner:", _flat_owner(params) is not None)
    opt.step()
    aux_loss = m.aux_loss()
    aux_loss.backward()
    aux.step()
    opt.zero_grad()
    aux.zero_grad()
