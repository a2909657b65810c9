"""Optimizer side of the training step (utils/engine.py:81-91; configure_optimizers,
models/Compression/common/model_utils.py:67-90).

* ``FusedAdam`` — torch.optim.Adam semantics (amsgrad=False, L2 weight decay), every parameter of
  a group updated by ONE HIP launch (tmae_adam_multi over a device table of tensors).
* ``clip_grad_norm_`` — torch.nn.utils.clip_grad_norm_ semantics; when every gradient lives in the
  training executor's flat buffer (the normal case after MCM's backward) it is one f64 reduction +
  one in-place scale over that buffer, with no host synchronisation.
* ``configure_optimizers`` — the reference split: Adam over everything but ``*.quantiles``, aux Adam
  over ``*.quantiles``.
"""
from __future__ import annotations

import torch

from . import _lib
from . import train_ops as T

CHUNK = 1024


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        for group in self.param_groups:
            for p in group["params"]:
                if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                    raise ValueError("FusedAdam needs contiguous f32 device parameters")
            n = sum(p.numel() for p in group["params"])
            dev = group["params"][0].device if group["params"] else None
            group["_m"] = torch.zeros(n, dtype=torch.float32, device=dev)
            group["_v"] = torch.zeros(n, dtype=torch.float32, device=dev)
            group["_step"] = 0
            group["_tab_key"] = None

    def _table(self, group, live):
        key = tuple((p.data_ptr(), p.grad.data_ptr()) for p in live)
        if group["_tab_key"] == key:
            return group["_tab"], group["_nchunks"]
        off, o = {}, 0
        for p in group["params"]:
            off[id(p)] = o
            o += p.numel()
        mb, vb = group["_m"], group["_v"]
        rows, chunk = [], 0
        for p in live:
            n = p.numel()
            rows.append([p.data_ptr(), p.grad.data_ptr(), mb[off[id(p)]:].data_ptr(), vb[off[id(p)]:].data_ptr(), n,
                         chunk])
            chunk += (n + CHUNK - 1) // CHUNK
        tab = torch.tensor(rows, dtype=torch.int64).to(mb.device)
        group["_tab"], group["_nchunks"], group["_tab_key"] = tab, chunk, key
        return tab, chunk

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            live = [p for p in group["params"] if p.grad is not None]
            if not live:
                continue
            for p in live:
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    raise ValueError("FusedAdam needs contiguous f32 gradients")
            group["_step"] += 1
            tab, nchunks = self._table(group, live)
            b1, b2 = group["betas"]
            _lib.call("tmae_adam_multi", tab.data_ptr(), len(live), nchunks, float(group["lr"]), float(b1), float(b2),
                      float(group["eps"]), float(group["weight_decay"]), group["_step"], None,
                      torch.cuda.current_stream().cuda_stream)
        return loss


def _flat_owner(params):
    """the flat gradient buffer when every gradient is a view of one executor buffer covering it exactly"""
    gs = [p.grad for p in params if p.grad is not None]
    if not gs:
        return None
    base = gs[0]._base
    if base is None or any(g._base is not base for g in gs):
        return None
    if sum(g.numel() for g in gs) != base.numel():
        return None
    return base


def clip_grad_norm_(parameters, max_norm, out=None):
    """torch.nn.utils.clip_grad_norm_ (L2): returns the total norm as a 0-d device tensor"""
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.zeros(())
    flat = _flat_owner(params)
    if flat is None:
        return torch.nn.utils.clip_grad_norm_(params, max_norm)
    res = out if out is not None else torch.empty(2, dtype=torch.float32, device=flat.device)
    T.grad_norm(flat, max_norm, res)
    T.scale_(flat, res[1:])
    return res[0]


def configure_optimizers(model, lr=1e-4, aux_lr=1e-4, fused=True):
    """reference model_utils.configure_optimizers (sorted names, quantiles to the aux optimizer)"""
    params = dict(model.named_parameters())
    main = sorted(n for n, p in params.items() if not n.endswith(".quantiles") and p.requires_grad)
    aux = sorted(n for n, p in params.items() if n.endswith(".quantiles") and p.requires_grad)
    cls = FusedAdam if fused else torch.optim.Adam
    return cls([params[n] for n in main], lr=lr), cls([params[n] for n in aux], lr=aux_lr)
