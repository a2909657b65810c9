"""Optimizer side of the training step (utils/engine.py:81-91; configure_optimizers,
models/Compression/common/model_utils.py:67-90).

* ``FusedAdam`` — torch.optim.Adam semantics (amsgrad=False, L2 weight decay, per-parameter step counts),
  every parameter of a group updated by ONE HIP launch (tmae_adam_multi over a device table of tensors).
  The moments live in one flat f32 buffer per group, the step counts in a device int32 array;
  ``state_dict()`` / ``load_state_dict()`` speak torch.optim.Adam's per-parameter format (``step``,
  ``exp_avg``, ``exp_avg_sq``), so a checkpoint written by the reference's ``save_model``
  (model_utils.py:30-55, torch Adam) resumes here and vice versa.
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


def bump_versions(params):
    """The update kernel writes parameters through raw pointers, which autograd's version counters do
    not see; the weight caches of the executors (bf16 casts, conv relayouts) are keyed on
    (data_ptr, _version), so every updated parameter gets its version advanced here."""
    ps = tuple(params)
    if ps:
        torch._C._autograd._unsafe_set_version_counter(ps, tuple(p._version + 1 for p in ps))


class _PinnedArena:
    """pinned host staging for launch tables built while a stream is being captured: neither a pageable H2D copy
    nor a pinned allocation may happen during a capture, so the pinned buffer is reserved before it
    (``reserve_capture_staging``) and handed out by a bump allocator.  The graph's copy nodes read their slices
    at every replay, so every capture gets a FRESH buffer (never a reset of the previous one, which a graph still
    alive would read) and the graph's owner keeps it alive.  ``epoch`` counts the captures: a table built inside
    capture e is filled only by that graph's copy node, so it is valid inside capture e and nowhere else
    (``table_usable``)."""

    def __init__(self):
        self.buf, self.off, self.epoch = None, 0, 0

    def reserve(self, nbytes):
        n = (int(nbytes) + 7) // 8
        self.buf = torch.empty(n, dtype=torch.int64).pin_memory()
        self.off = 0
        self.epoch += 1
        return self.buf

    def take(self, n):
        if self.buf is None or self.off + n > self.buf.numel():
            raise RuntimeError("launch table built during a HIP graph capture without enough pinned staging: call "
                               "optim.reserve_capture_staging() before capturing")
        v = self.buf[self.off:self.off + n]
        self.off += (n + 7) // 8 * 8  # 64-B aligned slices
        return v


_ARENA = _PinnedArena()


def reserve_capture_staging(nbytes=8 << 20):
    """a fresh pinned staging buffer for the launch tables built inside the NEXT graph capture; the caller (the
    graph's owner) keeps the returned buffer alive as long as the graph, whose copy nodes read it at every replay"""
    return _ARENA.reserve(nbytes)


def device_table(rows, device):
    """int64 rows -> a device table for a multi-tensor launch.  While a stream is being captured into a HIP graph
    the copy comes from the pinned staging arena (a pageable H2D copy or a pinned allocation cannot be captured);
    returns (table, capture epoch or None).  Pass the epoch to ``table_usable`` before reusing a cached table."""
    h = torch.tensor(rows, dtype=torch.int64).reshape(-1)
    if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
        p = _ARENA.take(h.numel())
        p.copy_(h)
        return p.to(device, non_blocking=True), _ARENA.epoch
    return h.to(device), None


def table_usable(epoch):
    """may a cached launch table built at capture ``epoch`` (None: built eagerly) be launched from now?  An eager
    table is filled when it is made.  A table built inside a capture holds its rows only once that graph's copy
    node has run, so it is reused only inside the same capture: not eagerly (before the first replay it is still
    uninitialised) and not in a later capture (a re-capture before any replay would read the same garbage)."""
    if epoch is None:
        return True
    return torch.cuda.is_current_stream_capturing() and epoch == _ARENA.epoch


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, L2 weight decay) with one HIP launch per group.

    Step counts are per parameter and live on the device (int32, advanced by the update launch itself), as
    torch.optim.Adam keeps ``state[p]["step"]`` per parameter: a parameter without a gradient at some step is
    skipped and keeps its count, exactly like torch's loop.  Nothing on the step path reads a host value that
    changes from step to step (the bias corrections come from the device counts), so the whole training step
    -- optimizer included -- can be captured into a HIP graph and replayed (engine.GraphedTrainStep).  The
    learning rate, betas, eps and weight decay are launch arguments: a graph bakes in the values it was
    captured with."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        for group in self.param_groups:
            for p in group["params"]:
                if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                    raise ValueError("FusedAdam needs contiguous f32 device parameters")
        self._flat = [self._new_flat(g) for g in self.param_groups]  # per group: [m, v, steps, offsets]
        self._bc = [self._new_bc(g) for g in self.param_groups]  # per group: 2 f32 bias corrections per parameter
        self._tabs = [None] * len(self.param_groups)

    @staticmethod
    def _new_bc(group):
        dev = group["params"][0].device if group["params"] else None
        return torch.zeros(2 * max(len(group["params"]), 1), dtype=torch.float32, device=dev)

    @staticmethod
    def _new_flat(group):
        off, o = {}, 0
        for i, p in enumerate(group["params"]):
            off[id(p)] = (o, i)
            o += p.numel()
        dev = group["params"][0].device if group["params"] else None
        z = torch.zeros(o, dtype=torch.float32, device=dev)
        steps = torch.zeros(max(len(group["params"]), 1), dtype=torch.int32, device=dev)
        return [z, torch.zeros_like(z), steps, off]

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        if hasattr(self, "_flat"):
            self._flat.append(self._new_flat(self.param_groups[-1]))
            self._bc.append(self._new_bc(self.param_groups[-1]))
            self._tabs.append(None)

    def _table(self, gi, live):
        key = tuple((p.data_ptr(), p.grad.data_ptr()) for p in live)
        hit = self._tabs[gi]
        if hit is not None and hit[0] == key and table_usable(hit[3]):
            return hit[1], hit[2]
        mb, vb, steps, off = self._flat[gi]
        bc = self._bc[gi]
        rows, owner, chunk = [], [], 0
        for t, p in enumerate(live):
            n = p.numel()
            o, i = off[id(p)]
            rows += [p.data_ptr(), p.grad.data_ptr(), mb[o:].data_ptr(), vb[o:].data_ptr(), n, chunk,
                     steps[i:].data_ptr(), bc[2 * i:].data_ptr()]
            nch = (n + CHUNK - 1) // CHUNK
            owner += [t] * nch
            chunk += nch
        tab, epoch = device_table(rows + owner, mb.device)  # the rows, then each chunk's row (tmae.h)
        self._tabs[gi] = (key, tab, chunk, epoch)
        return tab, chunk

    @torch.no_grad()
    def step(self, closure=None, grad_scale=None):
        """grad_scale: optional 1-element f32 device tensor every gradient is multiplied by inside the update
        (clip_grad_norm_'s factor left unapplied by clip_norm_deferred; the same f32 product scale_ would store)"""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            live = [p for p in group["params"] if p.grad is not None]
            if not live:
                continue
            for p in live:
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    raise ValueError("FusedAdam needs contiguous f32 gradients")
            tab, nchunks = self._table(gi, live)
            b1, b2 = group["betas"]
            _lib.call("tmae_adam_multi", tab.data_ptr(), len(live), nchunks, float(group["lr"]), float(b1), float(b2),
                      float(group["eps"]), float(group["weight_decay"]),
                      None if grad_scale is None else grad_scale.data_ptr(), torch.cuda.current_stream().cuda_stream)
            bump_versions(live)
        return loss

    # ------------------------------------------------------------------ checkpoints (torch.optim.Adam format)
    def state_dict(self):
        self.state.clear()
        for gi, group in enumerate(self.param_groups):
            mb, vb, steps, off = self._flat[gi]
            counts = steps.cpu().tolist()
            for p in group["params"]:
                (o, i), n = off[id(p)], p.numel()
                if counts[i] == 0:
                    continue  # torch Adam has no state for a parameter before its first step
                self.state[p] = {"step": torch.tensor(float(counts[i])), "exp_avg": mb[o:o + n].view_as(p).clone(),
                                 "exp_avg_sq": vb[o:o + n].view_as(p).clone()}
        try:
            return super().state_dict()
        finally:
            self.state.clear()

    def load_state_dict(self, state_dict):
        # torch moves per-parameter state to each parameter's device (the reference loads with
        # map_location="cpu", model_utils.py:14-17); the flat moments are rebuilt from it
        super().load_state_dict(state_dict)
        self._flat = [self._new_flat(g) for g in self.param_groups]
        self._bc = [self._new_bc(g) for g in self.param_groups]
        self._tabs = [None] * len(self.param_groups)
        for gi, group in enumerate(self.param_groups):
            mb, vb, steps, off = self._flat[gi]
            counts = [0] * steps.numel()
            for p in group["params"]:
                st = self.state.get(p)
                if not st:
                    continue
                (o, i), n = off[id(p)], p.numel()
                mb[o:o + n].copy_(st["exp_avg"].reshape(-1))
                vb[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                counts[i] = int(float(st["step"]))
            steps.copy_(torch.tensor(counts, dtype=torch.int32))
        self.state.clear()


def _flat_owner(params):
    """the flat gradient buffer when the gradients tile one executor buffer exactly: the same f32 storage,
    contiguous, disjoint, covering it (autograd detaches the views the HIP backward returns, so they are
    matched by storage and offsets, not by ``_base``)"""
    gs = [p.grad for p in params if p.grad is not None]
    if not gs:
        return None
    st = gs[0].untyped_storage()
    sp = st.data_ptr()
    if any(g.dtype != torch.float32 or not g.is_contiguous() or g.untyped_storage().data_ptr() != sp for g in gs):
        return None
    n = st.nbytes() // 4
    spans = sorted((g.storage_offset(), g.numel()) for g in gs)
    pos = 0
    for off, k in spans:
        if off != pos:
            return None
        pos += k
    if pos != n:
        return None
    return torch.empty(0, dtype=torch.float32, device=gs[0].device).set_(st, 0, (n,))


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


def clip_norm_deferred(parameters, max_norm, out):
    """clip_grad_norm_ with the scaling left to the optimizer: when every gradient lives in one flat buffer, writes
    out[0] = total norm, out[1] = min(1, max_norm / (norm + 1e-6)) and returns True without touching the gradients
    (pass out[1:] to FusedAdam.step(grad_scale=...)); otherwise clips in place like clip_grad_norm_ and returns
    False."""
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return False
    flat = _flat_owner(params)
    if flat is None:
        torch.nn.utils.clip_grad_norm_(params, max_norm)
        return False
    T.grad_norm(flat, max_norm, out)
    return True


def configure_optimizers(model, lr=1e-4, aux_lr=1e-4, fused=True):
    """reference model_utils.configure_optimizers (sorted names, quantiles to the aux optimizer)"""
    params = dict(model.named_parameters())
    main = sorted(n for n, p in params.items() if not n.endswith(".quantiles") and p.requires_grad)
    aux = sorted(n for n, p in params.items() if n.endswith(".quantiles") and p.requires_grad)
    cls = FusedAdam if fused else torch.optim.Adam
    return cls([params[n] for n in main], lr=lr), cls([params[n] for n in aux], lr=aux_lr)
