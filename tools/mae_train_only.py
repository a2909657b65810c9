"""The graphed MAE training step alone (bench.py's mae_train leg) for profiling: capture, 3 replays, a marker spin
kernel, then N timed replays; prints the wall time per step.  python tools/mae_train_only.py [N] [batch]"""
import sys
import time

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402
from textmae_amd import engine  # noqa: E402
from textmae_amd.optim import FusedAdam  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
m = textmae_amd.mae_vit_base_patch16_dec512d8b().cuda().train()
m.compute_dtype = torch.bfloat16
imgs = torch.randn(B, 3, 224, 224, generator=torch.Generator().manual_seed(3000)).cuda()
opt = FusedAdam([p for p in m.parameters() if p.requires_grad], lr=1.5e-4)
step = engine.GraphedMAEStep(m, opt, imgs, 0.75, warmup=2)
for _ in range(3):
    step(imgs)
torch.cuda.synchronize()
torch._C._cuda_sleep(1000)
t0 = time.perf_counter()
for _ in range(n):
    step(imgs)
torch.cuda.synchronize()
print(f"graphed MAE train step: {(time.perf_counter() - t0) / n * 1e3:.3f} ms wall at batch {B}")
