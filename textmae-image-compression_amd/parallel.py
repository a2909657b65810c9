"""Image-batch data parallelism for the training step (the DP that the reference's
training.py builds a DistributedSampler for but never initialises, training.py:122-129).

One process per GPU, ``torch.distributed`` backend "nccl" = RCCL over xGMI.  The model's backward
(mcm_train.py) produces every parameter gradient into ONE flat f32 buffer, in the order the reverse
pass finishes them (decoder first, patch embedding last).  ``GradSync`` cuts that buffer into
buckets and all-reduces each bucket as soon as the backward reports it final (``ready(upto)``), so
the collectives overlap the remaining backward kernels: the RCCL call is enqueued on the compute
stream's timeline (the process group's own stream waits for the point of the call), and
``finish()`` makes the compute stream wait for the last bucket -- no host synchronisation.

Bucket size: xGMI is point-to-point (7 links per GPU); a ring all-reduce moves 2(W-1)/W of a bucket
over each link, so buckets of ~64 MB keep every ring step long enough to run near link rate while
still giving the overlap several hand-off points per backward (804 MB of gradients -> ~13 buckets).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradSync:
    """``always_collective``: issue the collectives even in a one-rank group (by default a world of 1
    returns before them).  Tests use it to run the RCCL branch -- async ``AVG`` all-reduce per bucket,
    ``Work.wait()`` ordering against the compute stream -- on a single GPU."""

    def __init__(self, process_group=None, bucket_mb: float = 64.0, average: bool = True,
                 always_collective: bool = False, timing: bool = False):
        self.group = process_group
        self.bucket_elems = max(1, int(bucket_mb * (1 << 20) // 4))
        self.average = average
        self.always_collective = always_collective
        self.launched = 0  # collectives issued (tests check the buckets really went out)
        self.launched_in_backward = 0  # of those, issued by ready() while the backward was still running
        self.flat = None
        self._bounds = None
        self._next = 0
        self._work = []
        # timing (observability of the overlap, no host sync): HIP events on the compute stream at the first
        # bucket's launch point, at the end of the backward (finish() called) and after the last collective's
        # completion is ordered before the compute stream
        self.timing = timing
        self._ev = None
        self._first = None
        self._finishing = False

    def world(self):
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def capturable(self):
        """can a HIP graph hold this step's collectives?  RCCL's can (backend "nccl"); gloo's go through host memory"""
        if self.world() <= 1 and not (self.always_collective and dist.is_initialized()):
            return True  # no collective is issued
        return dist.get_backend(self.group) == "nccl"

    def _begin(self, flat):
        if self.flat is None or self.flat.data_ptr() != flat.data_ptr() or self.flat.numel() != flat.numel():
            n = flat.numel()
            self._bounds = list(range(0, n, self.bucket_elems)) + [n]
        self.flat = flat
        self._next = 0
        self._work = []
        self._first = None
        self.launched_in_backward = 0

    def _event(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream(self.flat.device))
        return e

    def _timed(self):
        """timing events on this backward: not inside a HIP graph capture (a captured step's overlap is read from an
        eager step of the same kernels, bench.py)"""
        return self.timing and self.flat is not None and self.flat.is_cuda and \
            not torch.cuda.is_current_stream_capturing()

    def attach(self, flat):
        """start a backward over `flat` (called by the executor before the first ready())"""
        self._begin(flat)

    def _launch(self, i):
        a, b = self._bounds[i], self._bounds[i + 1]
        t = self.flat[a:b]
        W = self.world()
        if W <= 1 and not (self.always_collective and dist.is_initialized()):
            return
        self.launched += 1
        if self._timed() and self._first is None:
            self._first = self._event()
        if dist.get_backend(self.group) == "nccl":
            # also under a HIP graph capture (engine.GraphedTrainStep): RCCL's kernels on the process group's stream
            # join the capture through its event wait on the compute stream, and Work.wait() below joins it back
            op = dist.ReduceOp.AVG if self.average else dist.ReduceOp.SUM
            self._work.append(dist.all_reduce(t, op=op, group=self.group, async_op=True))
        else:  # gloo (CPU rehearsal, or several ranks sharing one GPU in tests): SUM then scale
            if t.is_cuda and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("GradSync: a gloo all-reduce (host-staged) cannot be captured into a HIP graph")
            _host_all_reduce_sum(t, self.group)
            if self.average:
                t.div_(W)

    def ready(self, upto: int):
        """gradients [0, upto) of the flat buffer are final: launch every bucket they complete"""
        while self._next < len(self._bounds) - 1 and self._bounds[self._next + 1] <= upto:
            n0 = self.launched
            self._launch(self._next)
            if not self._finishing:
                self.launched_in_backward += self.launched - n0
            self._next += 1

    def finish(self):
        """launch the remaining buckets and order the compute stream after every collective"""
        timed = self._timed()
        end = self._event() if timed else None  # the backward's last kernel is enqueued before this point
        self._finishing = True
        try:
            self.ready(self._bounds[-1])
        finally:
            self._finishing = False
        for w in self._work:
            w.wait()
        self._work = []
        if timed:
            self._ev = (self._first, end, self._event(), len(self._bounds) - 1, self.flat.numel() * 4,
                        self.launched_in_backward)

    def last_timing(self):
        """the last backward's overlap numbers (synchronises on its events): ``allreduce_exposed_ms`` = end of the
        backward's kernels -> every collective complete on the compute stream's timeline; ``allreduce_issue_ms`` =
        first bucket's launch point -> end of the backward (how long the collectives ran under backward kernels);
        bucket count and bytes; how many buckets were issued from inside the backward"""
        if self._ev is None:
            return None
        first, end, done, nb, nbytes, inb = self._ev
        done.synchronize()
        return {"allreduce_exposed_ms": round(end.elapsed_time(done), 3),
                "allreduce_issue_ms": round(first.elapsed_time(end), 3) if first is not None else None,
                "buckets": nb, "bucket_bytes": self.bucket_elems * 4, "grad_bytes": nbytes,
                "buckets_issued_in_backward": inb}


def _host_all_reduce_sum(t, group):
    """gloo all-reduce of a tensor that may live on the GPU: staged through host memory (the device
    copy also orders the collective after every kernel that wrote `t` on the current stream)"""
    if not t.is_cuda:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return
    h = t.cpu()
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    t.copy_(h)


def broadcast_parameters(model, src: int = 0, group=None):
    """every rank starts from rank `src`'s weights (and buffers: the entropy models' CDF tables)"""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    staged = dist.get_backend(group) != "nccl"
    with torch.no_grad():
        for t in list(model.parameters()) + [b for b in model.buffers() if b.numel() > 0]:
            if staged and t.is_cuda:
                h = t.data.cpu()
                dist.broadcast(h, src=src, group=group)
                t.data.copy_(h)
            else:
                dist.broadcast(t.data, src=src, group=group)
    # the executors' weight caches are keyed on parameter versions, which these raw writes do not advance
    from .optim import bump_versions

    bump_versions(model.parameters())


def enable_data_parallel(model, process_group=None, bucket_mb: float = 64.0, always_collective: bool = False,
                         timing: bool = False):
    """attach a GradSync to `model` (MCM): its backward then all-reduces (averages) the gradients"""
    model.grad_sync = GradSync(process_group, bucket_mb, always_collective=always_collective, timing=timing)
    broadcast_parameters(model, group=process_group)
    return model.grad_sync
