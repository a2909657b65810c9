"""Which torch (ATen) operators does one eager MCM training step still launch, and from where?  The graphed step
replays them too (fills, copies, casts), each a ~4-5 us kernel.  torch.profiler over one eager step at the bench
config, ATen operators with a CUDA kernel under them, grouped by the innermost frames of our package.
    python tools/torch_ops_profile.py [batch]"""
import sys
from collections import Counter, defaultdict

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402
from textmae_amd import engine  # noqa: E402
from textmae_amd.optim import configure_optimizers  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
torch.manual_seed(0)
m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
m.compute_dtype = torch.bfloat16
m.distortion = "ssim+l1"
opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
crit = RateDistortionLoss(lmbda=1e-2)
imgs, scores = bench.synthetic_inputs(B, 256, 256, 2000, "cuda")
for _ in range(2):
    engine.train_step(m, crit, imgs, scores, opt, aux, clip_max_norm=1.0)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    engine.train_step(m, crit, imgs, scores, opt, aux, clip_max_norm=1.0)
    torch.cuda.synchronize()

# kernels launched under each ATen op (device time), keyed by the op and our innermost source frames
agg = defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if not ev.name.startswith("aten::") or ev.device_type.name != "CPU":
        continue
    kids = [k for k in ev.kernels] if hasattr(ev, "kernels") else []
    if not kids:
        continue
    frames = [f for f in (ev.stack or []) if "textmae-image-compression_amd" in f or "textmae_amd" in f]
    key = (ev.name, " <- ".join(f.split("/")[-1] for f in frames[:2]))
    agg[key][0] += len(kids)
    agg[key][1] += sum(k.duration for k in kids)
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
tot_n, tot_us = sum(v[0] for v in agg.values()), sum(v[1] for v in agg.values())
print(f"ATen kernels in one eager step: {tot_n}, {tot_us:.0f} us")
for (name, where), (n, us) in rows[:40]:
    print(f"{us:8.1f} us  x{n:4d}  {name:28s} {where}")
