"""Optimizer and data-parallel hand-off on the MI355X (the training call site, utils/engine.py:75-91).

* FusedAdam against torch.optim.Adam over several real MCM training steps (f32 and bf16 operands):
  the executors' weight caches must follow the in-place parameter updates;
* FusedAdam checkpoints in torch.optim.Adam's format (model_utils.py:9-55 save / resume);
* the DP bucket hand-off: every ``ready(upto)`` the HIP backward reports must come after the last write
  into gradients [0, upto) -- checked with a recording GradSync on one GPU, and with two ranks on
  cuda:0 over gloo, whose averaged gradients must equal a single-process full-batch backward and be
  bitwise identical to a run that defers every bucket to ``finish()``;
* the RCCL branch of GradSync (backend "nccl", async ``AVG`` all-reduce per bucket, ``Work.wait()``
  ordering) run for real in a one-rank group with the world-of-1 short-circuit bypassed: training steps
  bitwise equal to a run without data parallelism;
* ``bench.py --gpus 2`` without a launcher spawns its own two ranks.
"""
import io
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SMALL = dict(img_size=64, patch_size=16, encoder_embed_dim=64, encoder_depth=2, encoder_num_heads=2,
             decoder_embed_dim=64, decoder_depth=2, decoder_num_heads=2, latent_depth=192, hyperprior_depth=96,
             num_slices=12, num_keep_patches=16)


def _model(cfgd, seed, dt):
    import textmae_amd
    from oracle.mcm_oracle import MCMConfig, make_state_dict

    cfg = MCMConfig(**cfgd)
    m = textmae_amd.MCM(**cfg.kwargs())
    full = m.state_dict()
    full.update(make_state_dict(cfg, seed))
    m.load_state_dict(full)
    m = m.cuda().train()
    m.compute_dtype = dt
    return m, cfg


def _inputs(cfg, B, seed):
    rng = np.random.default_rng(seed)
    L = (cfg.img_size // cfg.patch_size) ** 2
    g = int(cfg.num_keep_patches ** 0.5)
    imgs = torch.from_numpy(rng.random((B, 3, cfg.img_size, cfg.img_size), dtype=np.float32))
    scores = torch.from_numpy(rng.random((B, L), dtype=np.float32))
    zn = torch.from_numpy(rng.uniform(-0.5, 0.5, (B, cfg.hyperprior_depth, g // 4, g // 4)).astype(np.float32))
    yn = torch.from_numpy(rng.uniform(-0.5, 0.5, (B, cfg.latent_depth, g, g)).astype(np.float32))
    return imgs, scores, zn, yn


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def _train_steps(m, opt, aux_opt, batches, crit):
    from textmae_amd import engine

    losses = []
    for imgs, scores, zn, yn in batches:
        out = engine.train_step(m, crit, imgs.cuda(), scores.cuda(), opt, aux_opt, clip_max_norm=1.0,
                                noise=(zn.cuda(), yn.cuda()))
        losses.append(float(out["loss"].detach()))
    torch.cuda.synchronize()
    return losses


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_adam_tracks_torch_adam(dt):
    """3 training steps: FusedAdam and torch.optim.Adam give the same losses and weights.  With stale
    weight caches (the update kernel writes through raw pointers) the FusedAdam run would keep
    forwarding the step-0 weights in bf16, and its losses would drift from the torch run."""
    from textmae_amd.optim import configure_optimizers
    from textmae_amd.rd_loss import RateDistortionLoss

    crit = RateDistortionLoss(lmbda=1e-2)
    m1, cfg = _model(SMALL, 21, dt)
    m2, _ = _model(SMALL, 21, dt)
    m1.distortion = m2.distortion = "ssim+l1"
    batches = [_inputs(cfg, 2, 100 + i) for i in range(3)]
    o1 = configure_optimizers(m1, lr=3e-3, aux_lr=1e-3, fused=True)
    o2 = configure_optimizers(m2, lr=3e-3, aux_lr=1e-3, fused=False)
    l1 = _train_steps(m1, *o1, batches, crit)
    l2 = _train_steps(m2, *o2, batches, crit)
    tol = 1e-4 if dt == torch.float32 else 2e-3
    assert np.allclose(l1, l2, rtol=tol), (l1, l2)
    # Adam moves every weight by at most ~lr per step: in f32 the two updates agree to a small part of that.
    # (Not checked in bf16: a last-ulp difference in an updated weight can flip its bf16 cast, and Adam's
    # normalised step turns the gradient noise on a near-zero gradient into up to ~lr per step.)
    if dt == torch.float32:
        atol = 5e-2 * 3e-3 * len(batches)
        p1, p2 = dict(m1.named_parameters()), dict(m2.named_parameters())
        bad = [(n, float((p1[n] - p2[n]).abs().max())) for n in p1 if float((p1[n] - p2[n]).abs().max()) > atol]
        assert not bad, bad[:10]
    # the eval executor after FusedAdam steps == a fresh model carrying the same weights
    import textmae_amd

    m1.eval()
    fresh = textmae_amd.MCM(**cfg.kwargs())
    fresh.load_state_dict(m1.state_dict())
    fresh = fresh.cuda().eval()
    fresh.compute_dtype = dt
    imgs, scores, _, _ = batches[0]
    with torch.no_grad():
        a = m1(imgs.cuda(), scores.cuda())["x_hat"]
        b = fresh(imgs.cuda(), scores.cuda())["x_hat"]
    assert torch.equal(a, b)


def test_fused_adam_checkpoint_roundtrip():
    """save_model / load_model (model_utils.py:9-55): the optimizer state goes through torch.save,
    comes back on the CPU (map_location="cpu") and the resumed run continues bit for bit; the state is
    torch.optim.Adam's format in both directions."""
    from textmae_amd.optim import FusedAdam
    from textmae_amd.rd_loss import RateDistortionLoss

    crit = RateDistortionLoss(lmbda=1e-2)
    m, cfg = _model(SMALL, 22, torch.float32)
    m.distortion = "none"
    batches = [_inputs(cfg, 2, 200 + i) for i in range(3)]
    main = [p for n, p in m.named_parameters() if not n.endswith(".quantiles")]
    aux = [m.entropy_bottleneck.quantiles]
    opt, aux_opt = FusedAdam(main, lr=1e-3), FusedAdam(aux, lr=1e-3)
    _train_steps(m, opt, aux_opt, batches[:2], crit)
    buf = io.BytesIO()
    torch.save({"model": m.state_dict(), "optimizer": opt.state_dict(), "aux_optimizer": aux_opt.state_dict()}, buf)
    buf.seek(0)
    ck = torch.load(buf, map_location="cpu", weights_only=True)
    assert set(ck["optimizer"]["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}

    m2, _ = _model(SMALL, 0, torch.float32)
    m2.distortion = "none"
    m2.load_state_dict(ck["model"])
    main2 = [p for n, p in m2.named_parameters() if not n.endswith(".quantiles")]
    opt2, aux2 = FusedAdam(main2, lr=1e-3), FusedAdam([m2.entropy_bottleneck.quantiles], lr=1e-3)
    opt2.load_state_dict(ck["optimizer"])
    aux2.load_state_dict(ck["aux_optimizer"])
    la = _train_steps(m, opt, aux_opt, batches[2:], crit)
    lb = _train_steps(m2, opt2, aux2, batches[2:], crit)
    assert la == lb
    for (n, p), q in zip(m.named_parameters(), m2.parameters()):
        assert torch.equal(p, q), n
    # a torch.optim.Adam checkpoint resumes in FusedAdam and the other way round
    tadam = torch.optim.Adam(main2, lr=1e-3)
    tadam.load_state_dict(opt2.state_dict())
    st = tadam.state_dict()
    opt3 = FusedAdam(main2, lr=1e-3)
    opt3.load_state_dict(st)
    s2, s3 = opt2.state_dict()["state"], opt3.state_dict()["state"]
    assert all(torch.equal(s2[k]["exp_avg"], s3[k]["exp_avg"]) and float(s2[k]["step"]) == float(s3[k]["step"])
               for k in s2)


class _Recorder:
    """GradSync stand-in: snapshots gflat[:upto] at every hand-off"""

    def __init__(self):
        self.snaps, self.uptos = [], []

    def attach(self, flat):
        self.flat = flat

    def ready(self, upto):
        self.uptos.append(upto)
        self.snaps.append(self.flat[:upto].clone())

    def finish(self):
        pass


@pytest.mark.parametrize("geom", ["small", "vitb"])
def test_backward_ready_points_are_final(geom):
    """every gradient below a ready() offset is final when ready() is called: a bucket launched there
    must not see a later write (mcm_train.py _ready / parallel.GradSync)"""
    from textmae_amd.rd_loss import RateDistortionLoss

    if geom == "small":
        m, cfg = _model(SMALL, 23, torch.float32)
    else:
        import textmae_amd
        from oracle.mcm_oracle import MCMConfig

        torch.manual_seed(0)
        cfg = MCMConfig(img_size=256, num_keep_patches=144)
        m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
        m.compute_dtype = torch.bfloat16
    m.distortion = "ssim+l1"
    rec = _Recorder()
    m.grad_sync = rec
    imgs, scores, zn, yn = _inputs(cfg, 2, 300)
    out = m(imgs.cuda(), scores.cuda(), noise=(zn.cuda(), yn.cuda()))
    loss = RateDistortionLoss(lmbda=1e-2)(out, imgs.cuda())["loss"]
    m.zero_grad(set_to_none=True)
    loss.backward()
    torch.cuda.synchronize()
    final = rec.flat
    assert rec.uptos == sorted(rec.uptos) and rec.uptos[-1] == final.numel()
    assert len(rec.uptos) >= 2 * (m.decoder_depth + m.encoder_depth)
    stale = [(u, int((s != final[:u]).sum())) for u, s in zip(rec.uptos, rec.snaps) if not torch.equal(s, final[:u])]
    assert not stale, stale[:5]


# ------------------------------------------------------------------------------ two ranks on cuda:0
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import textmae_amd  # noqa: F401
        from textmae_amd.parallel import GradSync, enable_data_parallel
        from textmae_amd.rd_loss import RateDistortionLoss

        crit = RateDistortionLoss(lmbda=1e-2)
        m, cfg = _model(SMALL, 24 + rank, torch.float32)  # rank 1 starts from other weights: broadcast fixes it
        m.distortion = "ssim+l1"
        imgs, scores, zn, yn = _inputs(cfg, 4, 400)
        half = slice(2 * rank, 2 * rank + 2)

        def grads(sync):
            m.grad_sync = sync
            m.zero_grad(set_to_none=True)
            out = m(imgs[half].cuda(), scores[half].cuda(), noise=(zn[half].cuda(), yn[half].cuda()))
            crit(out, imgs[half].cuda())["loss"].backward()
            torch.cuda.synchronize()
            return torch.cat([p.grad.reshape(-1).cpu() for p in m.parameters() if p.requires_grad])

        sync = enable_data_parallel(m, bucket_mb=0.05)  # small buckets: many early launches
        g_early = grads(sync)
        nb = len(sync._bounds) - 1

        class Deferred(GradSync):
            """every bucket waits for finish()"""
            armed = False

            def ready(self, upto):
                if self.armed:
                    super().ready(upto)

            def finish(self):
                self.armed = True
                super().finish()

        g_deferred = grads(Deferred(bucket_mb=0.05))
        q.put((rank, g_early.numpy(), g_deferred.numpy(), nb))  # plain arrays: no shared-memory fds to outlive us
    except BaseException as e:  # report instead of leaving the parent waiting on the queue
        q.put((rank, None, repr(e)[:2000], 0))
        raise
    finally:
        dist.destroy_process_group()


def test_dp_two_ranks_match_full_batch():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=150) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    errs = [b for _, a, b, _ in res if a is None]
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs)
    (_, e0, d0, nb), (_, e1, d1, _) = [(r, torch.from_numpy(a), torch.from_numpy(b), n) for r, a, b, n in res]
    assert nb > 10
    assert torch.equal(e0, e1) and torch.equal(e0, d0) and torch.equal(d0, d1)

    # single process, full batch of 4, rank 0's weights
    from textmae_amd.rd_loss import RateDistortionLoss

    m, cfg = _model(SMALL, 24, torch.float32)
    m.distortion = "ssim+l1"
    imgs, scores, zn, yn = _inputs(cfg, 4, 400)
    out = m(imgs.cuda(), scores.cuda(), noise=(zn.cuda(), yn.cuda()))
    RateDistortionLoss(lmbda=1e-2)(out, imgs.cuda())["loss"].backward()
    torch.cuda.synchronize()
    ref = torch.cat([p.grad.reshape(-1).cpu() for p in m.parameters() if p.requires_grad])
    rel2 = float((e0.double() - ref.double()).norm() / ref.double().norm())
    assert rel2 < 1e-5, rel2
    assert _rel(e0, ref) < 1e-4


def test_bench_two_ranks_gloo_prints_one_line():
    """the driver's N>1 launch line (torch.distributed.run, one rank per GPU) rehearsed with two
    ranks on one GPU over gloo: one JSON line, value aggregated over both ranks"""
    import json

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--steps", "2", "--warmup", "1", "--batch", "4", "--train-steps", "1", "--train-warmup", "1",
           "--train-batch", "2", "--kernel-reps", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["train"]["global_batch"] == 4


# ------------------------------------------------------------------------------ RCCL branch, one rank
def _nccl_w1_worker(port, geom, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import textmae_amd
        from textmae_amd.optim import configure_optimizers
        from textmae_amd.parallel import enable_data_parallel
        from textmae_amd.rd_loss import RateDistortionLoss

        assert dist.get_backend() == "nccl"
        crit = RateDistortionLoss(lmbda=1e-2)

        def make():
            if geom == "small":
                m, cfg = _model(SMALL, 31, torch.float32)
            else:
                from oracle.mcm_oracle import MCMConfig

                torch.manual_seed(0)
                cfg = MCMConfig(img_size=256, num_keep_patches=144)
                m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
                m.compute_dtype = torch.bfloat16
            m.distortion = "ssim+l1"
            return m, cfg

        res = {}
        for mode in ("plain", "rccl"):
            m, cfg = make()
            sync = enable_data_parallel(m, bucket_mb=8.0 if geom == "vitb" else 0.05,
                                        always_collective=True, timing=True) if mode == "rccl" else None
            opt, aux = configure_optimizers(m, lr=1e-3, aux_lr=1e-3, fused=True)
            batches = [_inputs(cfg, 2, 500 + i) for i in range(2)]
            losses = _train_steps(m, opt, aux, batches, crit)
            # one more backward, kept: the gradients themselves
            imgs, scores, zn, yn = _inputs(cfg, 2, 600)
            out = m(imgs.cuda(), scores.cuda(), noise=(zn.cuda(), yn.cuda()))
            crit(out, imgs.cuda())["loss"].backward()
            torch.cuda.synchronize()
            g = torch.cat([p.grad.reshape(-1).cpu() for p in m.parameters() if p.requires_grad])
            w = torch.cat([p.detach().reshape(-1).float().cpu() for p in m.parameters()])
            res[mode] = (losses, g.numpy(), w.numpy(), sync.launched if sync is not None else 0)
            if sync is not None:
                res["timing"] = sync.last_timing()
        q.put(res)
    except BaseException as e:  # report instead of leaving the parent waiting on the queue
        q.put({"error": repr(e)[:2000]})
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("geom", ["small", "vitb"])
def test_rccl_grad_sync_one_rank_bitwise(geom):
    """GradSync's RCCL path executes (nccl process group of one rank, short-circuit bypassed): the
    bucketed async AVG all-reduces issued from inside the backward and the Work.wait() before the
    optimizer leave losses, gradients and post-step weights bitwise equal to a run without DP"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_w1_worker, args=(_port(), geom, q))
    p.start()
    res = q.get(timeout=170)
    p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert p.exitcode == 0
    (l0, g0, w0, _), (l1, g1, w1, launched) = res["plain"], res["rccl"]
    assert launched > 10, launched  # three backwards' worth of buckets really went through RCCL
    # the overlap is real: most buckets leave from inside the backward (ready() hand-offs), and the first one's
    # launch point on the compute stream precedes the backward's end
    t = res["timing"]
    assert t["buckets_issued_in_backward"] >= t["buckets"] // 2, t
    assert t["allreduce_issue_ms"] is not None and t["allreduce_issue_ms"] > 0, t
    assert t["allreduce_exposed_ms"] >= 0, t
    assert l0 == l1
    assert np.array_equal(g0, g1)
    assert np.array_equal(w0, w1)


def _nccl_graph_worker(port, q):
    """one-rank RCCL group: the captured DP step (GraphedTrainStep holding GradSync's bucketed all-reduces) against
    eager DP steps (the same GradSync, always_collective) on the same batches and noise"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from textmae_amd import engine
        from textmae_amd.optim import configure_optimizers
        from textmae_amd.parallel import enable_data_parallel
        from textmae_amd.rd_loss import RateDistortionLoss

        crit = RateDistortionLoss(lmbda=1e-2)
        res = {}
        for mode in ("eager", "graph"):
            m, cfg = _model(SMALL, 32, torch.bfloat16)
            m.distortion = "ssim+l1"
            sync = enable_data_parallel(m, bucket_mb=0.05, always_collective=True)
            opt, aux = configure_optimizers(m, lr=2e-3, aux_lr=1e-3, fused=True)
            batches = [_inputs(cfg, 2, 800 + i) for i in range(4)]
            cu = lambda b: tuple(t.cuda() for t in b)  # noqa: E731
            if mode == "eager":
                losses = _train_steps(m, opt, aux, batches, crit)
                info = {}
            else:
                imgs, scores, zn, yn = cu(batches[0])
                n0 = sync.launched
                g = engine.GraphedTrainStep(m, crit, opt, aux, imgs, scores, clip_max_norm=1.0, warmup=1,
                                            noise=(zn, yn))
                nb = len(sync._bounds) - 1
                info = {"buckets": nb, "captured": sync.launched - n0 - nb, "in_backward": sync.launched_in_backward}
                losses = [None]  # step 0 is the warm-up step inside the constructor
                for b in batches[1:]:
                    imgs, scores, zn, yn = cu(b)
                    losses.append(float(g(imgs, scores, noise=(zn, yn))["loss"]))
                n1 = sync.launched
                torch.cuda.synchronize()
                info["host_launches_during_replays"] = sync.launched - n1
            w = torch.cat([p.detach().reshape(-1).float().cpu() for p in m.parameters()])
            res[mode] = (losses, w.numpy(), info)
        q.put(res)
    except BaseException as e:  # report instead of leaving the parent waiting on the queue
        q.put({"error": repr(e)[:2000]})
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_graphed_train_step_one_rank_bitwise():
    """the DP training step as ONE HIP graph: GradSync's RCCL all-reduces (one-rank nccl group, short-circuit
    bypassed) are captured from inside the backward (every bucket, most of them before the backward ends) and
    replayed with the step; losses and post-step weights bitwise equal to eager DP steps"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_graph_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=170)
    p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert p.exitcode == 0
    (le, we, _), (lg, wg, info) = res["eager"], res["graph"]
    assert info["buckets"] > 4 and info["captured"] == info["buckets"], info
    assert info["in_backward"] >= info["buckets"] // 2, info
    assert lg[1:] == le[1:], (lg, le)
    assert np.array_equal(we, wg)


def test_bench_spawns_ranks_without_launcher():
    """``python bench.py --gpus 2`` with no torch.distributed launcher: bench starts two ranks itself
    (before any GPU call in the parent) and prints one line for the whole job"""
    import json

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "2",
           "--warmup", "1", "--batch", "4", "--train-steps", "1", "--train-warmup", "1", "--train-batch", "2",
           "--no-roofline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["train"]["global_batch"] == 4


def test_fused_adam_partial_gradients_match_torch():
    """per-parameter step counts (torch.optim.Adam's state[p]["step"]): a parameter without a gradient at some
    step is skipped and keeps its count, so the bias corrections of the two parameters diverge exactly as in
    torch's loop; the state_dict carries the per-parameter counts"""
    from textmae_amd.optim import FusedAdam

    torch.manual_seed(3)
    init = [torch.randn(1000, device="cuda"), torch.randn(37, device="cuda")]
    grads = [[torch.randn(1000, device="cuda"), torch.randn(37, device="cuda")] for _ in range(4)]
    mask = [(1, 1), (1, 0), (1, 0), (0, 1)]  # which parameter has a gradient at each step
    runs = []
    for cls in (FusedAdam, torch.optim.Adam):
        ps = [torch.nn.Parameter(t.clone()) for t in init]
        kw = dict(foreach=False) if cls is torch.optim.Adam else {}
        opt = cls(ps, lr=1e-2, weight_decay=0.01, **kw)
        for g, mk in zip(grads, mask):
            for p, gi, on in zip(ps, g, mk):
                p.grad = gi.clone() if on else None
            opt.step()
        runs.append((ps, opt.state_dict()))
    (pa, sa), (pb, sb) = runs
    for a, b in zip(pa, pb):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), float((a - b).abs().max())
    assert [float(sa["state"][i]["step"]) for i in (0, 1)] == [3.0, 2.0]
    assert [float(sb["state"][i]["step"]) for i in (0, 1)] == [3.0, 2.0]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_graphed_train_step_bitwise(dt):
    """engine.GraphedTrainStep: the whole training step (forward, RateDistortionLoss, aux loss, HIP backward,
    clip_grad_norm_, both FusedAdam steps, zero_grad) captured once as a HIP graph and replayed per batch gives
    losses and post-step weights bitwise equal to eager engine.train_step on the same batches and noise; an
    eager forward after the replays sees the replayed weights (version counters advanced)"""
    from textmae_amd import engine
    from textmae_amd.optim import configure_optimizers
    from textmae_amd.rd_loss import RateDistortionLoss

    crit = RateDistortionLoss(lmbda=1e-2)
    m1, cfg = _model(SMALL, 23, dt)
    m2, _ = _model(SMALL, 23, dt)
    m1.distortion = m2.distortion = "ssim+l1"
    batches = [_inputs(cfg, 2, 300 + i) for i in range(4)]
    o1 = configure_optimizers(m1, lr=3e-3, aux_lr=1e-3, fused=True)
    o2 = configure_optimizers(m2, lr=3e-3, aux_lr=1e-3, fused=True)
    cu = lambda b: tuple(t.cuda() for t in b)  # noqa: E731
    imgs, scores, zn, yn = cu(batches[0])
    # construction = one eager warm-up step on batch 0, then the capture
    g = engine.GraphedTrainStep(m1, crit, *o1, imgs, scores, clip_max_norm=1.0, warmup=1, noise=(zn, yn))
    la = []
    for b in batches[1:]:
        imgs, scores, zn, yn = cu(b)
        out = g(imgs, scores, noise=(zn, yn))
        la.append(float(out["loss"]))
    lb = _train_steps(m2, *o2, batches, crit)[1:]
    assert la == lb, (la, lb)
    for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p, q), n
    m1.eval()
    m2.eval()
    imgs, scores, _, _ = cu(batches[0])
    with torch.no_grad():
        assert torch.equal(m1(imgs, scores)["x_hat"], m2(imgs, scores)["x_hat"])


def test_graphed_train_step_lr_change_before_first_replay():
    """a learning-rate change BEFORE the first replay re-captures at once: the launch tables the first capture
    built (relayout, Adam) were never filled (their copy nodes had not run), so the second capture and an eager
    forward in between must build their own.  Losses and weights stay bitwise equal to eager steps with the same
    schedule (a reused, unfilled table would launch on garbage pointers)."""
    from textmae_amd import engine
    from textmae_amd.optim import configure_optimizers
    from textmae_amd.rd_loss import RateDistortionLoss

    crit = RateDistortionLoss(lmbda=1e-2)
    m1, cfg = _model(SMALL, 25, torch.bfloat16)
    m2, _ = _model(SMALL, 25, torch.bfloat16)
    m1.distortion = m2.distortion = "ssim+l1"
    batches = [_inputs(cfg, 2, 700 + i) for i in range(3)]
    o1 = configure_optimizers(m1, lr=3e-3, aux_lr=1e-3, fused=True)
    o2 = configure_optimizers(m2, lr=3e-3, aux_lr=1e-3, fused=True)
    cu = lambda b: tuple(t.cuda() for t in b)  # noqa: E731
    imgs, scores, zn, yn = cu(batches[0])
    g = engine.GraphedTrainStep(m1, crit, *o1, imgs, scores, clip_max_norm=1.0, warmup=1, noise=(zn, yn))
    # an eager training forward between the capture and the first replay (tables of the capture unfilled)
    out = m1(imgs, scores, noise=(zn, yn))
    del out
    for grp in o1[0].param_groups:
        grp["lr"] = 1e-3
    la = []
    for b in batches[1:]:
        imgs, scores, zn, yn = cu(b)
        la.append(float(g(imgs, scores, noise=(zn, yn))["loss"]))
    lb = _train_steps(m2, *o2, batches[:1], crit)
    for grp in o2[0].param_groups:
        grp["lr"] = 1e-3
    lb = _train_steps(m2, *o2, batches[1:], crit)
    assert la == lb, (la, lb)
    for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p, q), n


def test_graphed_train_step_device_noise_and_lr_change():
    """without injected noise the graph draws training noise from torch's graph-safe generator (a fresh draw
    per replay); changing the learning rate re-captures the step"""
    from textmae_amd import engine
    from textmae_amd.optim import configure_optimizers
    from textmae_amd.rd_loss import RateDistortionLoss

    crit = RateDistortionLoss(lmbda=1e-2)
    m, cfg = _model(SMALL, 24, torch.bfloat16)
    m.distortion = "ssim+l1"
    opt, aux = configure_optimizers(m, lr=1e-3, aux_lr=1e-3, fused=True)
    imgs, scores, _, _ = (t.cuda() for t in _inputs(cfg, 2, 400))
    g = engine.GraphedTrainStep(m, crit, opt, aux, imgs, scores)
    bpp = []
    for _ in range(3):
        bpp.append(float(g(imgs, scores)["bpp_loss"]))
    first = g.graph
    assert len(set(bpp)) == 3 and all(np.isfinite(bpp)), bpp
    for grp in opt.param_groups:
        grp["lr"] = 5e-4
    g(imgs, scores)
    assert g.graph is not first
    st = opt.state_dict()["state"]
    assert {float(v["step"]) for v in st.values()} == {5.0}
