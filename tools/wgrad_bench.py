"""Micro-benchmark of the training step's ViT weight gradients (train_ops.wgrad, split-K TN GEMM + fixed-order
reduce) at the bench shapes, alone on the GPU: out[M][N] = dY^T X with K = tokens (encoder 64 x 145, decoder
64 x 257), bias column sums included.  Per shape and slot divisor: us per call (20 calls replayed in a HIP graph)
and TFLOP/s.     python tools/wgrad_bench.py [slot_div ...]"""
import json
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import train_ops as T  # noqa: E402

SHAPES = {  # name: (M = out features, N = in features, K = token rows)
    "enc_qkv": (2304, 768, 64 * 145), "enc_proj": (768, 768, 64 * 145), "enc_fc1": (3072, 768, 64 * 145),
    "enc_fc2": (768, 3072, 64 * 145), "dec_qkv": (1536, 512, 64 * 257), "dec_fc1": (2048, 512, 64 * 257),
    "dec_fc2": (512, 2048, 64 * 257),
}


def timed(run):
    run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            run()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 20 * 1e-3)
    return best


def main():
    divs = [int(v) for v in sys.argv[1:]] or [1, 2]
    out = {}
    for name, (M, N, K) in SHAPES.items():
        dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)
        x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
        w = torch.empty(M, N, device="cuda")
        b = torch.empty(M, device="cuda")
        for sd in divs:
            t = timed(lambda: T.wgrad(dy, x, M, N, K, w, torch.bfloat16, bias=b, slot_div=sd))
            out[f"{name}_sd{sd}"] = {"us": round(t * 1e6, 1), "tflops": round(2.0 * M * N * K / t / 1e12, 1)}
            print(name, sd, out[f"{name}_sd{sd}"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
