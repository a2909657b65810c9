"""Micro-benchmark of the LIC latent partial sums (mcm._slices pre(): the first slice-stack convs' latent part,
384 input channels, f32 output, no bias) at the bench shapes: batch 64, 12x12, bf16.  Per shape: us per launch
and TFLOP/s from 20 launches replayed in a HIP graph, for the halo conv (tmae_conv3x3) and tmae_lic_latent.
    python tools/psum_bench.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops  # noqa: E402


def timed(run):
    run()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run()
    torch.cuda.current_stream().wait_stream(side)
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
    B, H, M, S, c0, dt = 64, 12, 384, 12, 224, torch.bfloat16
    Mp = B * H * H
    out = {}
    x = torch.randn(2, Mp, M, device="cuda").to(dt)
    Pw = 3 * S * c0
    y = torch.empty(Mp, Pw, device="cuda")
    # halo conv: [mean | lrp] on x[1] (2 problems) and scale on x[0], n columns per problem
    for name, n in {"halo_slice": c0, "halo_6to11": 6 * c0}.items():
        w = (torch.randn(3, n, 9 * M, device="cuda") / (9 * M) ** 0.5).to(dt)

        def run():
            ops.conv3x3(x[1], M, M, B, H, H, w, None, y, Pw, n, dt, y_f32=True, nb=(1, 2),
                        strides={"w": (0, n * 9 * M), "y": (0, S * c0)})
            ops.conv3x3(x[0], M, M, B, H, H, w[2], None, y[:, 2 * S * c0:], Pw, n, dt, y_f32=True)

        t = timed(run)
        out[name] = {"us": round(t * 1e6, 1), "tflops": round(2.0 * 3 * Mp * n * 9 * M / t / 1e12, 1)}
        print(name, out[name], flush=True)
    nfs = c0 // 16
    w = torch.randn(3 * S, c0, M, 3, 3, device="cuda") / (9 * M) ** 0.5
    wpk = torch.stack([ops.pack_lic_stack_weight(wi) for wi in w]).contiguous()
    for name, (i0, i1) in {"latent_slice": (1, 2), "latent_6to11": (6, 12), "latent_all": (0, 12)}.items():
        def run():
            ops.lic_latent(B, H, [x[1], x[1], x[0]], M, M, wpk, nfs, wpk[0].numel(), [0, S * nfs, 2 * S * nfs],
                           i0 * nfs, i1 * nfs, y, Pw)

        t = timed(run)
        n = (i1 - i0) * c0
        out[name] = {"us": round(t * 1e6, 1), "tflops": round(2.0 * 3 * Mp * n * 9 * M / t / 1e12, 1)}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
