"""Train / validation loops — counterparts of reference utils/engine.py:30-219 with the same call
pattern on the model (``model(samples, total_scores)``, ``criterion(out_net, samples)``,
``model.aux_loss()``, loss.backward(), clip_grad_norm_(model.parameters(), clip), optimizer.step(),
aux_loss.backward(), aux_optimizer.step(), zero_grad x2) and the same metric names.

What differs (MI355X-side, not semantics):
  * the six per-step metric all-reduces of the reference (engine.py:117-122, each behind a blocking
    ``.item()``) are ONE 6-element all-reduce, read back once per step;
  * the gradient all-reduce of data parallelism runs inside the backward (parallel.GradSync);
  * with ``fused=True`` clip_grad_norm_ / Adam are the flat-buffer HIP kernels (optim.py).
Logging (MetricLogger / TensorBoard) is out of scope.
"""
from __future__ import annotations

import torch

from . import distributed
from .optim import clip_grad_norm_

METRICS = ("loss", "L1_loss", "ssim_loss", "vgg_loss", "bpp_loss", "aux_loss")


def train_step(model, criterion, samples, total_scores, optimizer, aux_optimizer, clip_max_norm=1.0, accum_iter=1,
               step_now=True, noise=None):
    """one iteration of the reference loop body (utils/engine.py:72-91); returns the device losses"""
    out_net = model(samples, total_scores, noise=noise) if noise is not None else model(samples, total_scores)
    out_criterion = criterion(out_net, samples)
    out_criterion["loss"] = out_criterion["loss"] / accum_iter
    aux_loss = model.aux_loss() / accum_iter
    if step_now:
        out_criterion["loss"].backward()
        if clip_max_norm > 0:
            clip_grad_norm_(model.parameters(), clip_max_norm)
        optimizer.step()
        aux_loss.backward()
        aux_optimizer.step()
        optimizer.zero_grad()
        aux_optimizer.zero_grad()
    out_criterion["aux_loss"] = aux_loss
    return out_criterion


def train_one_epoch(model, criterion, train_dataloader, optimizer, aux_optimizer, epoch, clip_max_norm=1.0,
                    accum_iter=1, log=None):
    """utils/engine.py:30-156 (without MetricLogger / TensorBoard); returns the per-metric averages"""
    model.train()
    device = next(model.parameters()).device
    optimizer.zero_grad()
    aux_optimizer.zero_grad()
    sums = torch.zeros(len(METRICS), dtype=torch.float64)
    n = 0
    for i, (samples, _ori_shape, total_scores) in enumerate(train_dataloader):
        samples = samples.to(device, non_blocking=True)
        total_scores = total_scores.to(device, non_blocking=True)
        out = train_step(model, criterion, samples, total_scores, optimizer, aux_optimizer, clip_max_norm, accum_iter,
                         step_now=(i + 1) % accum_iter == 0)
        vals = torch.stack([out[k].detach().float().reshape(()) for k in METRICS]).cpu().double()
        reduced = distributed.all_reduce_mean_many(vals.tolist())
        sums += torch.tensor(reduced, dtype=torch.float64)
        n += 1
        if log is not None:
            log(epoch, i, dict(zip(METRICS, reduced)))
    return {k: round(float(v) / max(n, 1), 7) for k, v in zip(METRICS, sums)}


@torch.no_grad()
def val_one_epoch(epoch, val_dataloader, model, criterion):
    """utils/engine.py:159-219: eval mode, no_grad, autocast (bf16 operands on MI355X)"""
    model.eval()
    device = next(model.parameters()).device
    sums = torch.zeros(len(METRICS), dtype=torch.float64)
    n = 0
    for samples, _ori_shape, total_scores in val_dataloader:
        samples = samples.to(device)
        total_scores = total_scores.to(device)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out_net = model(samples, total_scores)
            out = criterion(out_net, samples)
            out["aux_loss"] = model.aux_loss()
        sums += torch.tensor([float(out[k]) for k in METRICS], dtype=torch.float64)
        n += 1
    avg = distributed.all_reduce_mean_many((sums / max(n, 1)).tolist())
    return {k: round(v, 2) for k, v in zip(METRICS, avg)}
