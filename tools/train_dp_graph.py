"""The graphed training step with and without the one-rank RCCL gradient all-reduce (bench.py's
`train.grad_allreduce.graphed` leg against its plain `train` leg), for kernel traces of one replay of each:
capture, 3 replays, then N timed replays; prints the wall time per step.
  python tools/train_dp_graph.py {plain|dp} [N] [bucket_mb]"""
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402
from textmae_amd import engine  # noqa: E402
from textmae_amd.optim import configure_optimizers  # noqa: E402
from textmae_amd.parallel import enable_data_parallel  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "dp"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
bucket = float(sys.argv[3]) if len(sys.argv) > 3 else 64.0
B = 64
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
m.compute_dtype = torch.bfloat16
m.distortion = "ssim+l1"
if mode == "dp":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    enable_data_parallel(m, bucket_mb=bucket, always_collective=True)
opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
crit = RateDistortionLoss(lmbda=1e-2)
imgs, scores = bench.synthetic_inputs(B, 256, 256, 2000, "cuda")
g = engine.GraphedTrainStep(m, crit, opt, aux, imgs, scores, clip_max_norm=1.0, warmup=1)
for _ in range(3):
    g(imgs, scores)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    g(imgs, scores)
torch.cuda.synchronize()
print(f"{mode} graphed train step: {(time.perf_counter() - t0) / n * 1e3:.2f} ms wall at batch {B}, bucket {bucket} MB")
if mode == "dp":
    dist.destroy_process_group()
