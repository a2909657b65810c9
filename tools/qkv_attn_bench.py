"""Fused qkv + attention (tmae_qkv_attn_fwd) against the unfused qkv GEMM + attention core at the bench shapes:
back-to-back launches between HIP events, median of 5 runs of 20.   usage: python tools/qkv_attn_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import textmae_amd  # noqa: E402
from textmae_amd import ops  # noqa: E402


def timeit(fn, reps=20, runs=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(runs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    textmae_amd.load_library()
    bf = torch.bfloat16
    for name, B, T, H, dh in (("enc", 64, 145, 12, 64), ("dec", 64, 257, 16, 32), ("enc_k64", 64, 65, 12, 64)):
        D = H * dh
        x = torch.randn(B * T, D, device="cuda").to(bf)
        w = (torch.randn(3 * D, D, device="cuda") / D ** 0.5).to(bf)
        b = torch.randn(3 * D, device="cuda") * 0.1
        qkv = torch.empty(B * T, 3 * D, device="cuda", dtype=bf)
        o = torch.empty(B * T, D, device="cuda", dtype=bf)
        s = dh ** -0.5
        t_gemm = timeit(lambda: ops.linear(x, w, b, bf, out=qkv))
        t_core = timeit(lambda: ops.mha(qkv, B, T, H, dh, s, bf, out=o))
        t_fused = timeit(lambda: ops.qkv_attn(x, w, b, B, T, H, dh, s, bf, out=o))
        gf = (2 * B * T * D * 3 * D + 4 * B * H * T * T * dh) / 1e9
        print(f"{name}: qkv GEMM {t_gemm:.1f} us + core {t_core:.1f} us = {t_gemm + t_core:.1f} us | fused "
              f"{t_fused:.1f} us ({gf / t_fused * 1e3:.0f} TF/s, {gf / t_fused * 1e3 / 2500:.3f} of peak)", flush=True)


if __name__ == "__main__":
    main()
