"""Benchmark: images/s of MCM encode + rate + decode (BASELINE.json metric) on MI355X.

One step = one MCM.forward (eval: masking ids on device, ViT-B/16 encoder, LIC hyperprior with
EntropyBottleneck + 12-slice GaussianConditional likelihoods, ViT decoder, unpatchify) over a batch
of 64 synthetic 256x256 RGB images with K=144 kept patches, bf16 MFMA operands (f32 accumulate,
f32 entropy models).  The forward is replayed as a HIP graph; inputs are resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Multi-GPU: images are independent, so every rank runs its own batch of 64 with no
collective on the data path ("weak" scaling); the barrier + max-over-ranks timing follows the
driver contract.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec encode+decode+rate, ViT-B 256×256 batch64, 1/2/4/8 MI355X"
FWD_GFLOP_PER_IMG = 61.48        # BASELINE.md §2, config 2 (K=144)
TRAIN_GFLOP_PER_IMG = 184.4      # fwd + bwd = 3x fwd
PEAK_BF16 = 2.5e15               # MI355X_MICROARCH.md: dense bf16 MFMA
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--keep", type=int, default=144)
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--train-steps", type=int, default=10, help="training steps timed after the inference run")
    ap.add_argument("--train-warmup", type=int, default=3)
    ap.add_argument("--train-batch", type=int, default=64)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--backend", default="nccl", help="process-group backend (nccl = RCCL; gloo for a one-GPU rehearsal)")
    return ap.parse_args()


def synthetic_inputs(batch, img, L, seed, device):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(batch, 3, img, img, generator=g)
    mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    x = (x - mean) / std  # the train transform's Normalize (utils/dataloader.py:61)
    s = torch.rand(batch, L, generator=torch.Generator().manual_seed(seed + 1))
    return x.to(device), s.to(device)


def time_kernel(fn, reps):
    """average duration of one launch, HIP events on the stream the kernel is launched on"""
    st = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def dominant_kernel_roofline(model, batch, reps, dtype):
    """Encoder MLP fc1 GEMM (M = 64*145, N = 3072, K = 768, GELU epilogue): the single launch
    that carries the most FLOPs of the step (12 per forward, each 2*M*N*K)."""
    from textmae_amd import ops

    blk = model.encoder_blocks[0]
    T = model.num_keep_patches + 1
    M, N, K = batch * T, blk.mlp.fc1.out_features, blk.mlp.fc1.in_features
    x = torch.randn(M, K, device="cuda").to(dtype)
    w = blk.mlp.fc1.weight.detach().to(dtype).contiguous()
    b = blk.mlp.fc1.bias.detach()
    out = torch.empty(M, N, device="cuda", dtype=dtype)
    t = time_kernel(lambda: ops.linear(x, w, b, dtype, act=ops.ACT_GELU, out=out), reps)
    flops = 2.0 * M * N * K
    ach = flops / t / 1e12
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_fc1_gemm.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    plan = ops.gemm_plan(M, N, K, dtype)
    return {"kernel": "%s enc fc1+GELU (M=%d,N=%d,K=%d)" % (plan, M, N, K), "bound": "mfma",
            "achieved": round(ach, 2), "peak": PEAK_BF16 / 1e12, "unit": "TFLOP/s", "frac": round(ach * 1e12 / PEAK_BF16, 4),
            "traffic": traffic, "avg_launch_us": round(t * 1e6, 2), "flops_per_launch": flops}


def train_bench(model, args, rank, world, dev, barrier):
    """the reference training step (utils/engine.py:72-91): forward, RateDistortionLoss (SSIM + L1 +
    bpp; VGG needs a weight download), aux loss, backward (HIP reverse pass; for world > 1 the RCCL
    gradient all-reduce runs inside it, bucketed), clip_grad_norm_(1.0), Adam, aux backward, aux Adam"""
    from textmae_amd import engine
    from textmae_amd.optim import configure_optimizers
    from textmae_amd.parallel import enable_data_parallel
    from textmae_amd.rd_loss import RateDistortionLoss

    model.train()
    model.distortion = "ssim+l1"
    if world > 1:
        enable_data_parallel(model)
    opt, aux_opt = configure_optimizers(model, lr=1e-4, aux_lr=1e-4, fused=True)
    crit = RateDistortionLoss(lmbda=1e-2)
    L = model.encoder_embed.num_patches
    imgs, scores = synthetic_inputs(args.train_batch, args.img, L, 2000 + rank, dev)

    def step():
        return engine.train_step(model, crit, imgs, scores, opt, aux_opt, clip_max_norm=1.0)

    for _ in range(args.train_warmup):
        out = step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.train_steps):
        out = step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    ips = world * args.train_batch * args.train_steps / el
    return {"metric": "training images/s (fwd + bwd + clip + 2x Adam" + (", RCCL grad all-reduce" if world > 1 else "")
            + ")", "value": round(ips, 2), "unit": "images/s", "ms_per_step": round(el / args.train_steps * 1e3, 3),
            "steps": args.train_steps, "warmup": args.train_warmup, "per_gpu_batch": args.train_batch,
            "global_batch": args.train_batch * world, "parallelism": f"dp{world}", "dtype": "bf16",
            "loss_last": round(float(out["loss"].detach()), 6), "step_mfma_frac": round(ips * TRAIN_GFLOP_PER_IMG * 1e9 /
                                                                             (world * PEAK_BF16), 4),
            "hip_graph": False}


def cpu_baseline(img, keep, seconds):
    """The oracle (CPU restatement, fp32) on the host cores: a bounded 2-image sample of the workload."""
    from oracle.mcm_oracle import MCMConfig, make_state_dict, mcm_forward

    cfg = MCMConfig(img_size=img, num_keep_patches=keep)
    sd = make_state_dict(cfg, 0)
    x, s = synthetic_inputs(2, img, (img // 16) ** 2, 0, "cpu")
    n = 0
    t0 = time.perf_counter()
    while True:
        mcm_forward(sd, cfg, x, s)
        n += 2
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(n / el, 3), "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} images ({n // 2} oracle forwards of 2 x 256x256, K=144, fp32) in {el:.1f}s"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    import textmae_amd

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    model = textmae_amd.MCM(img_size=args.img, num_keep_patches=args.keep).to(dev).eval()
    model.compute_dtype = dtype
    model.distortion = "none"  # metric = encode + rate + decode; forward_loss is reported separately
    L = model.encoder_embed.num_patches
    imgs, scores = synthetic_inputs(args.batch, args.img, L, 1000 + rank, dev)

    graph = None
    with torch.no_grad():
        if args.no_graph:
            def step():
                model(imgs, scores)
        else:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    model(imgs, scores)
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                model(imgs, scores)

            def step():
                graph.replay()

        for _ in range(args.warmup):
            step()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        roof = dominant_kernel_roofline(model, args.batch, args.kernel_reps, dtype) if rank == 0 else None

    train = None
    if not args.no_train and args.train_steps > 0:
        graph = None
        train = train_bench(model, args, rank, world, dev, barrier)

    value = world * args.batch * args.steps / el
    rec = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded uniform RGB, "
        "ImageNet-normalised; uniform patch scores; seeded random-init weights)",
        "config": {"workload": "MCM forward eval: ids+ViT-B/16 enc (K=144 of 256 patches) + LIC hyperprior + "
                   "EB/GC rates + ViT dec + unpatchify", "img_size": args.img, "num_keep_patches": args.keep,
                   "per_gpu_batch": args.batch, "global_batch": args.batch * world, "parallelism": f"replicas x{world}",
                   "hip_graph": not args.no_graph},
        "step_mfma_frac": round(value * FWD_GFLOP_PER_IMG * 1e9 / (world * PEAK_BF16), 4),
        "roofline": roof,
    }
    if train is not None:
        rec["train"] = train
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.img, args.keep, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
