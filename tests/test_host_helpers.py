"""Call-site counterparts (CPU): optimizer split, batched metric all-reduce over a gloo process group
(world size 2, the N>1 host path), RateDistortionLoss arithmetic around the device bpp."""
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_configure_optimizers_split(tmae):
    from textmae_amd.model_utils import configure_optimizers

    m = tmae.MCM(img_size=64, encoder_embed_dim=64, encoder_depth=1, encoder_num_heads=2, decoder_embed_dim=32,
                 decoder_depth=1, decoder_num_heads=1, latent_depth=64, hyperprior_depth=32, num_slices=4,
                 num_keep_patches=16)
    opt, aux = configure_optimizers(m, SimpleNamespace(learning_rate=1e-4, aux_learning_rate=1e-3))
    n_main = sum(p.numel() for g in opt.param_groups for p in g["params"])
    n_aux = sum(p.numel() for g in aux.param_groups for p in g["params"])
    assert n_aux == m.entropy_bottleneck.quantiles.numel()
    assert n_main + n_aux == sum(p.numel() for p in m.parameters() if p.requires_grad)
    assert aux.param_groups[0]["lr"] == 1e-3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import textmae_amd  # noqa: F401
    from textmae_amd import distributed as D

    vals = [float(rank + i) for i in range(6)]
    out = D.all_reduce_mean_many(vals)
    q.put((rank, D.get_rank(), D.get_world_size(), out))
    dist.destroy_process_group()


def test_all_reduce_mean_many_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, r2, world, out in res:
        assert r2 == rank and world == 2
        assert out == pytest.approx([0.5 + i for i in range(6)])


def test_distributed_helpers_single_process(tmae):
    from textmae_amd import distributed as D

    assert D.get_rank() == 0 and D.get_world_size() == 1
    assert D.all_reduce_mean(3.5) == 3.5


def test_bench_rejects_gpus_world_size_mismatch():
    """bench.py --gpus N under a launcher that started a different WORLD_SIZE exits non-zero before any GPU
    call, instead of printing a line for the wrong world"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
