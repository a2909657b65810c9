"""Where the host's time goes in a graphed training step (host blocked ~22 ms of a ~31 ms
step).  Captures bench.py's one-rank training step, then times, per call, the host side of data.next()-like
input copies, graph.replay() and bump_versions separately, with the weight gradients on the side stream (the
default) and, in a second model, all on the compute stream.  Prints one JSON line per mode.
    python tools/replay_host.py [steps] [batch] [modes: side,noside]"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402
from textmae_amd import engine  # noqa: E402
from textmae_amd.optim import bump_versions, configure_optimizers  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
modes = (sys.argv[3] if len(sys.argv) > 3 else "side").split(",")


def run(mode):
    torch.manual_seed(0)
    m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
    m.compute_dtype = torch.bfloat16
    m.distortion = "ssim+l1"
    opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
    crit = RateDistortionLoss(lmbda=1e-2)
    imgs, scores = bench.synthetic_inputs(B, 256, 256, 2000, "cuda")
    if mode == "noside":  # one eager step builds the executor; then its weight gradients stay on the compute stream
        engine.train_step(m, crit, imgs, scores, opt, aux, clip_max_norm=1.0)
        m._train_exec._side = None
    g = engine.GraphedTrainStep(m, crit, opt, aux, imgs, scores, clip_max_norm=1.0, warmup=1)
    for _ in range(3):
        g(imgs, scores)
    torch.cuda.synchronize()
    t_copy = t_rep = t_bump = 0.0
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        g.samples.copy_(imgs, non_blocking=True)
        g.total_scores.copy_(scores, non_blocking=True)
        b = time.perf_counter()
        g.graph.replay()
        c = time.perf_counter()
        bump_versions(g.params)
        d = time.perf_counter()
        t_copy += b - a
        t_rep += c - b
        t_bump += d - c
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return {"mode": mode, "steps": n, "batch": B, "wall_ms_per_step": round(wall / n * 1e3, 3),
            "host_ms_per_step": round(host / n * 1e3, 3), "copy_ms": round(t_copy / n * 1e3, 3),
            "replay_ms": round(t_rep / n * 1e3, 3), "bump_ms": round(t_bump / n * 1e3, 3)}


for md in modes:
    print(json.dumps(run(md)), flush=True)
