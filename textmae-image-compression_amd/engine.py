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
from .optim import FusedAdam, clip_grad_norm_, clip_norm_deferred


def _clip_buffer(optimizer):
    """the persistent [norm, factor] f32 pair of this optimizer's deferred clip (allocated outside any capture)"""
    buf = getattr(optimizer, "_clip_buf", None)
    if buf is None:
        dev = next(p.device for g in optimizer.param_groups for p in g["params"])
        buf = optimizer._clip_buf = torch.empty(2, dtype=torch.float32, device=dev)
    return buf

def _drain_watchdog(group):
    """Return once the process group's watchdog holds no pending work: ``_wait_for_pending_works`` blocks until
    its work list is empty (the GPU must have finished them, so the device is synchronised first)."""
    import torch.distributed as dist

    torch.cuda.synchronize()
    pg = group if group is not None else dist.group.WORLD
    pg._wait_for_pending_works()


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
        scale = None
        if clip_max_norm > 0:
            if isinstance(optimizer, FusedAdam):
                # the clip factor goes into the Adam update (g * s, the product the in-place scale would store):
                # one pass over the 805 MB gradient buffer less; the gradients are zeroed below either way
                buf = _clip_buffer(optimizer)
                if clip_norm_deferred(model.parameters(), clip_max_norm, buf):
                    scale = buf[1:]
            else:
                clip_grad_norm_(model.parameters(), clip_max_norm)
        if scale is not None:
            optimizer.step(grad_scale=scale)
        else:
            optimizer.step()
        aux_loss.backward()
        aux_optimizer.step()
        optimizer.zero_grad()
        aux_optimizer.zero_grad()
    out_criterion["aux_loss"] = aux_loss
    return out_criterion


class GraphedTrainStep:
    """The loop body of utils/engine.py:72-91 (``train_step``) captured ONCE into a HIP graph and replayed per
    batch: forward (HIP kernels, device noise from torch's graph-safe generator), RateDistortionLoss, aux loss,
    the HIP backward, clip_grad_norm_, both FusedAdam steps and zero_grad are one ``graph.replay()``, so the host
    enqueues one launch per step instead of ~2500.

    What makes the step capturable: the library never allocates or synchronises; the optimizer's step counts
    and bias corrections live on the device (optim.FusedAdam); launch tables built during capture come from
    pinned memory (optim.device_table); the gradient buffer is persistent.  Construction runs ``warmup`` eager
    training steps on the first batch (ordinary optimizer steps: lazy workspaces and tables are created outside
    the capture), then captures one more step without running it.

    Each call copies the batch into the graph's static input tensors, replays, and advances the parameters'
    version counters (the update kernel writes through raw pointers; the executors' weight caches are keyed on
    the versions, so an eager forward after replays re-lays out the new weights).  The learning rates, betas,
    eps and weight decays are baked into the graph: when any of them changes, the step is captured again.
    Data parallelism over RCCL is captured too: GradSync's bucketed all-reduces are issued from inside the captured
    backward, so every replay runs them on the process group's stream under the remaining backward kernels, joined
    before clip / Adam (one ``graph.replay()`` per step at any world size, like the reference's one loop body,
    utils/engine.py:75-91).  The RCCL communicator exists before the capture (the eager warm-up step's
    collectives).  A gloo group (host-staged all-reduce) is refused: use ``train_step`` there."""

    def __init__(self, model, criterion, optimizer, aux_optimizer, samples, total_scores, clip_max_norm=1.0,
                 warmup=1, noise=None):
        sync = getattr(model, "grad_sync", None)
        if sync is not None and not sync.capturable():
            raise ValueError("GraphedTrainStep: a gloo gradient all-reduce (host-staged) is not capturable; use "
                             "engine.train_step, or the nccl (RCCL) backend whose collectives the graph holds")
        if not samples.is_cuda:
            raise ValueError("GraphedTrainStep needs device inputs")
        self.model, self.criterion = model, criterion
        self.optimizer, self.aux_optimizer = optimizer, aux_optimizer
        self.clip_max_norm = clip_max_norm
        self.samples = samples.detach().clone()
        self.total_scores = total_scores.detach().clone()
        # injected quantisation noise (parity tests): static tensors refreshed per call like the batch
        self.noise = tuple(t.detach().clone() for t in noise) if noise is not None else None
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.graph, self.out = None, None
        self._capture(warmup)

    def _hyper(self):
        return tuple((g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"])
                     for o in (self.optimizer, self.aux_optimizer) for g in o.param_groups)

    def _step(self):
        return train_step(self.model, self.criterion, self.samples, self.total_scores, self.optimizer,
                          self.aux_optimizer, self.clip_max_norm, noise=self.noise)

    def _capture(self, warmup):
        self.graph, self.out = None, None
        cur = torch.cuda.current_stream(self.samples.device)
        side = torch.cuda.Stream(device=self.samples.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._step()
        cur.wait_stream(side)
        self.optimizer.zero_grad()
        self.aux_optimizer.zero_grad()
        # every weight cache stale at capture time, so the graph always carries the per-step weight re-layout
        from .optim import bump_versions, reserve_capture_staging

        bump_versions(self.params)
        self._staging = reserve_capture_staging()  # the graph's copy nodes read it at every replay
        sync = getattr(self.model, "grad_sync", None)
        mode = "global"
        if sync is not None and (sync.world() > 1 or sync.always_collective):
            # the warm-up step's RCCL works sit in the process group's watchdog until it sees them complete; it
            # queries their end events, recorded on the process group's stream -- which the capture below turns
            # into a capturing stream, where such a query fails (hipErrorCapturedEvent) and takes the watchdog
            # down.  By construction: block until the watchdog has retired every pending work (collectives issued
            # during the capture are never handed to it), and capture in thread-local mode so that a query from
            # the watchdog's thread cannot invalidate the capture either.
            _drain_watchdog(sync.group)
            mode = "thread_local"
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=mode):
            out = self._step()
        self.graph, self.out = g, out
        self._hyper_at_capture = self._hyper()

    def __call__(self, samples, total_scores, noise=None):
        """one training step on (samples, total_scores); returns the step's device losses (static tensors,
        overwritten by the next call)"""
        if (noise is None) != (self.noise is None):
            raise ValueError("GraphedTrainStep: noise must be given at every call iff it was given at capture")
        if self._hyper() != self._hyper_at_capture:
            self._capture(0)
        self.samples.copy_(samples, non_blocking=True)
        self.total_scores.copy_(total_scores, non_blocking=True)
        if noise is not None:
            for dst, src in zip(self.noise, noise):
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        from .optim import bump_versions

        bump_versions(self.params)
        return self.out


class GraphedMAEStep:
    """MaskedAutoencoderViT pre-training step (models_mae.py:216-220 under autograd + an optimizer step) captured
    once into a HIP graph, replayed per batch: zero_grad, forward (masking noise from torch's graph-safe generator,
    or a static noise tensor refreshed per call), masked-MSE loss, the HIP backward (mae_train.py) and the FusedAdam
    update.  Same capture rules as GraphedTrainStep (device step counts, pinned launch tables, persistent gradient
    buffer); a changed learning rate re-captures.  Returns the step's loss (a static device tensor)."""

    def __init__(self, model, optimizer, imgs, mask_ratio=0.75, warmup=1, noise=None):
        if not imgs.is_cuda:
            raise ValueError("GraphedMAEStep needs device inputs")
        self.model, self.optimizer, self.mask_ratio = model, optimizer, mask_ratio
        self.imgs = imgs.detach().float().clone()
        self.noise = noise.detach().float().clone() if noise is not None else None
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.graph, self.loss = None, None
        self._capture(warmup)

    def _hyper(self):
        return tuple((g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]) for g in self.optimizer.param_groups)

    def _step(self):
        self.optimizer.zero_grad()
        loss, _, _ = self.model(self.imgs, self.mask_ratio, noise=self.noise)
        loss.backward()
        self.optimizer.step()
        return loss.detach()

    def _capture(self, warmup):
        from .optim import bump_versions, reserve_capture_staging

        self.graph, self.loss = None, None
        cur = torch.cuda.current_stream(self.imgs.device)
        side = torch.cuda.Stream(device=self.imgs.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._step()
        cur.wait_stream(side)
        self.optimizer.zero_grad()
        bump_versions(self.params)
        self._staging = reserve_capture_staging()  # the graph's copy nodes read it at every replay
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = self._step()
        self.graph, self.loss = g, loss
        self._hyper_at_capture = self._hyper()

    def __call__(self, imgs, noise=None):
        if (noise is None) != (self.noise is None):
            raise ValueError("GraphedMAEStep: noise must be given at every call iff it was given at capture")
        if self._hyper() != self._hyper_at_capture:
            self._capture(0)
        self.imgs.copy_(imgs, non_blocking=True)
        if noise is not None:
            self.noise.copy_(noise, non_blocking=True)
        self.graph.replay()
        from .optim import bump_versions

        bump_versions(self.params)
        return self.loss


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
