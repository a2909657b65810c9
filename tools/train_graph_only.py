"""The graphed training step alone (bench.py's one-rank train leg) for profiling: capture, 3 replays, a marker
spin kernel, then N timed replays; prints the wall time per step.  python tools/train_graph_only.py [N] [batch]"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402
from textmae_amd import engine  # noqa: E402
from textmae_amd.optim import configure_optimizers  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
m.compute_dtype = torch.bfloat16
opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
crit = RateDistortionLoss(lmbda=1e-2)
imgs, scores = bench.synthetic_inputs(B, 256, 256, 2000, "cuda")
g = engine.GraphedTrainStep(m, crit, opt, aux, imgs, scores, clip_max_norm=1.0, warmup=1)
for _ in range(3):
    g(imgs, scores)
torch.cuda.synchronize()
torch._C._cuda_sleep(1000)
t0 = time.perf_counter()
for _ in range(n):
    g(imgs, scores)
torch.cuda.synchronize()
print(f"graphed train step: {(time.perf_counter() - t0) / n * 1e3:.2f} ms wall at batch {B}")
