"""Process-group helpers — counterparts of reference models/Compression/common/distributed.py:5-33.

One process per GPU; backend "nccl" is RCCL on ROCm.  `all_reduce_mean_many` replaces the
reference's six back-to-back blocking scalar all-reduces per step (utils/engine.py:117-122) with one
6-element all-reduce.
"""
import torch
import torch.distributed as dist


def is_dist_avail_and_initialized():
    return dist.is_available() and dist.is_initialized()


def get_rank():
    return dist.get_rank() if is_dist_avail_and_initialized() else 0


def get_world_size():
    return dist.get_world_size() if is_dist_avail_and_initialized() else 1


def all_reduce_mean(x):
    return all_reduce_mean_many([x])[0]


def all_reduce_mean_many(values):
    """mean over ranks of a list of python floats, in ONE collective"""
    world = get_world_size()
    if world <= 1:
        return list(values)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    t /= world
    return t.tolist()
