"""Attention-core micro-benchmark at the bench shapes (batch 64): encoder T=145, 12 heads x 64;
decoder T=257, 16 heads x 32 (or the shapes given as name=B,T,H,dh arguments).  Forward and backward;
MFMA utilisation = algorithmic flops (4 B H T^2 dh fwd, 2.5x that bwd incl. recompute) / time / 2.5 PF."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops, train_ops  # noqa: E402

PEAK = 2.5e15


def ev(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps * 1e-3)
    return best


def main():
    out = {}
    dt = torch.bfloat16
    shapes = {"enc": (64, 145, 12, 64), "dec": (64, 257, 16, 32)}
    if len(sys.argv) > 1:  # name=B,T,H,dh ...
        shapes = {a.split("=")[0]: tuple(int(v) for v in a.split("=")[1].split(",")) for a in sys.argv[1:]}
    for name, (B, T, H, dh) in shapes.items():
        D = H * dh
        qkv = torch.randn(B * T, 3 * D, device="cuda").to(dt)
        o = torch.empty(B * T, D, device="cuda", dtype=dt)
        lse = torch.empty(B * H * T, device="cuda")
        do = torch.randn(B * T, D, device="cuda").to(dt)
        dq = torch.empty_like(qkv)
        fl = 4.0 * B * H * T * T * dh
        res = {}
        t = ev(lambda: ops.mha(qkv, B, T, H, dh, dh ** -0.5, dt, out=o))
        res["fwd_us"] = round(t * 1e6, 1)
        res["fwd_mfma_frac"] = round(fl / t / PEAK, 4)
        train_ops.mha_lse(qkv, B, T, H, dh, dh ** -0.5, dt, o, lse)
        t = ev(lambda: train_ops.mha_bwd(qkv, o, do, lse, dq, B, T, H, dh, dh ** -0.5, dt))
        res["bwd_us"] = round(t * 1e6, 1)
        res["bwd_mfma_frac"] = round(2.5 * fl / t / PEAK, 4)
        out[name] = res
        print(name, res, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
