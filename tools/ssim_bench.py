"""SSIM + L1 forward and backward (distortion.hip) at the training shape (64 x 3 x 256^2), back-to-back launches
between HIP events, median of 5 runs of 10.   usage: python tools/ssim_bench.py  (TMAE_LIB= for a variant)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import textmae_amd  # noqa: E402,F401
from textmae_amd import _lib  # noqa: E402
from textmae_amd.ops import _stream  # noqa: E402


def timeit(fn, reps=10, runs=5):
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
    g = torch.Generator().manual_seed(0)
    x = torch.rand(64, 3, 256, 256, generator=g).cuda()
    y = (x + 0.1 * torch.randn(64, 3, 256, 256, generator=g).cuda()).clamp(0, 1)
    P, H, W = 192, 256, 256
    h = torch.empty(5 * P * H * (W - 10), device="cuda")
    d = torch.empty(3 * P * (H - 10) * (W - 10), device="cuda")
    v = torch.empty(3 * P * H * (W - 10), device="cuda")
    part = torch.empty(2048, dtype=torch.float64, device="cuda")
    out = torch.empty(2, device="cuda")
    gout = torch.tensor([0.7, 1.3], device="cuda")
    gx = torch.empty_like(x)
    fwd = lambda: _lib.call("tmae_distortion_fwd", x.data_ptr(), y.data_ptr(), P, H, W, h.data_ptr(), d.data_ptr(),
                            part.data_ptr(), out.data_ptr(), _stream())
    bwd = lambda: _lib.call("tmae_distortion_bwd", x.data_ptr(), y.data_ptr(), P, H, W, d.data_ptr(), v.data_ptr(),
                            gout.data_ptr(), gx.data_ptr(), _stream())
    tf, tb = timeit(fwd), timeit(bwd)
    print(f"ssim+l1 fwd {tf:.1f} us  bwd {tb:.1f} us  loss {out.tolist()}  gx_sum {float(gx.double().sum()):.6e}",
          flush=True)


if __name__ == "__main__":
    main()
