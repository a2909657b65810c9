"""Data-parallel plumbing on CPU: world_size-2 gloo process group (127.0.0.1), the same GradSync /
broadcast / metric all-reduce code the GPU training step runs over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import textmae_amd  # noqa: F401
        from textmae_amd import distributed as tdist
        from textmae_amd.parallel import GradSync, broadcast_parameters

        # bucketed averaging, buckets completed out of alignment with the ready() points
        n = 10_000
        flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
        gs = GradSync(bucket_mb=1024 * 4 / (1 << 20))  # 1024-element buckets
        gs.attach(flat)
        launched = []
        for upto in (0, 700, 1024, 5000, 5001, 9999):
            gs.ready(upto)
            launched.append(gs._next)
        launched_before_finish = launched
        gs.finish()
        ok_avg = torch.allclose(flat, torch.arange(n, dtype=torch.float32) * 1.5)

        # rank 0's weights everywhere
        m = torch.nn.Linear(4, 3)
        with torch.no_grad():
            m.weight.fill_(float(rank + 7))
        broadcast_parameters(m)
        ok_bcast = bool((m.weight == 7.0).all())

        # one collective for the six metrics
        vals = tdist.all_reduce_mean_many([rank * 1.0, 2.0, rank * 4.0, 0.0, 1.0, -rank * 1.0])
        q.put((rank, ok_avg, launched_before_finish, ok_bcast, vals))
    finally:
        dist.destroy_process_group()


def test_gradsync_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, ok_avg, launched, ok_bcast, vals in res:
        assert ok_avg, rank
        # a bucket goes out as soon as the ready prefix covers it; the partial last one waits for finish()
        assert launched == [0, 0, 1, 4, 4, 9]
        assert ok_bcast
        assert vals == pytest.approx([0.5, 2.0, 2.0, 0.0, 1.0, -0.5])


def test_train_oracle_matches_forward_oracle():
    """the autograd-faithful oracle computes the same values as the golden-pinned forward oracle"""
    import numpy as np

    from oracle.mcm_oracle import MCMConfig, make_state_dict, mcm_forward
    from oracle.train_oracle import mcm_forward_train

    cfg = MCMConfig(img_size=64, encoder_embed_dim=64, encoder_depth=1, encoder_num_heads=2, decoder_embed_dim=64,
                    decoder_depth=1, decoder_num_heads=2, latent_depth=192, hyperprior_depth=96, num_keep_patches=16)
    sd = make_state_dict(cfg, 3)
    rng = np.random.default_rng(4)
    imgs = torch.from_numpy(rng.random((2, 3, 64, 64), dtype=np.float32))
    sc = torch.from_numpy(rng.random((2, 16), dtype=np.float32))
    zn = torch.from_numpy(rng.uniform(-.5, .5, (2, 96, 1, 1)).astype(np.float32))
    yn = torch.from_numpy(rng.uniform(-.5, .5, (2, 192, 4, 4)).astype(np.float32))
    a = mcm_forward(sd, cfg, imgs, sc, zn, yn)
    b = mcm_forward_train(sd, cfg, imgs, sc, zn, yn)
    assert torch.equal(a.x_hat, b[0]) and torch.equal(a.y_likelihood, b[1]) and torch.equal(a.z_likelihood, b[2])


def test_lower_bound_backward_semantics():
    from oracle.train_oracle import lower_bound

    x = torch.tensor([0.05, 0.2, 0.05, 0.2], requires_grad=True)
    y = lower_bound(x, 0.11)
    y.backward(torch.tensor([1.0, 1.0, -1.0, -1.0]))
    # below the bound the gradient passes only when it is negative (compressai LowerBoundFunction)
    assert x.grad.tolist() == [0.0, 1.0, -1.0, -1.0]
