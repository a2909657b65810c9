"""Micro-benchmark of the hyperprior's implicit-GEMM 3x3 convs (h_a layers 3-5, h_s layers 1-4: the ConvSrc
launches of tmae_conv3x3) at the bench shapes (batch 64, latent grid 12x12, bf16), each also at half its input
channels (the half-K time is what a 2-way split of K would run per split) and as a dense GEMM of the same
M x N x K (ops.linear: what the implicit-conv row source costs).  20 launches replayed from one HIP
graph, best of 5, us per launch.
usage: python tools/hyper_conv_bench.py [name ...]"""
import json
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops  # noqa: E402

SHAPES = {  # name: (cin, cout, input grid, stride, problems, pixel shuffle)
    "ha3_336_288_s2": (336, 288, 12, 2, 1, False), "ha4_288_240": (288, 240, 6, 1, 1, False),
    "ha5_240_192_s2": (240, 192, 6, 2, 1, False), "hs1_192_240": (192, 240, 3, 1, 2, False),
    "hs2_240_1152_ps": (240, 1152, 3, 1, 2, True), "hs3_288_336": (288, 336, 6, 1, 2, False),
    "hs4_336_1536_ps": (336, 1536, 6, 1, 2, True),
}


def bench(cin, cout, H, stride, nb, ps, B=64, dt=torch.bfloat16):
    Ho = (H - 1) // stride + 1
    x = torch.randn(B * H * H, cin, device="cuda").to(dt)
    w = (torch.randn(nb, cout, 9 * cin, device="cuda") / (9 * cin) ** 0.5).to(dt)
    b = torch.randn(nb, cout, device="cuda")
    y = torch.empty(nb, B * Ho * Ho * cout, device="cuda", dtype=dt)
    strides = {"w": (0, cout * 9 * cin), "b": (0, cout), "y": (0, B * Ho * Ho * cout), "x1": (0, 0)}

    def run():
        ops.conv3x3(x, cin, cin, B, H, H, w, b, y, cout // 4 if ps else cout, cout, dt, stride=stride,
                    act=ops.ACT_GELU, pixel_shuffle=ps, nb=(1, nb), strides=strides)

    run()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run()
    torch.cuda.current_stream().wait_stream(side)
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
    fl = 2.0 * nb * B * Ho * Ho * cout * 9 * cin
    return {"us": round(best * 1e6, 1), "tflops": round(fl / best / 1e12, 1)}


def bench_dense(cin, cout, H, stride, nb, B=64, dt=torch.bfloat16):
    """the same M x N x K as one plain token GEMM (ops.linear, dense rows): the ConvSrc gather's cost"""
    Ho = (H - 1) // stride + 1
    M, K = nb * B * Ho * Ho, 9 * cin
    x = torch.randn(M, K, device="cuda").to(dt)
    w = (torch.randn(cout, K, device="cuda") / K ** 0.5).to(dt)
    b = torch.randn(cout, device="cuda")
    y = torch.empty(M, cout, device="cuda", dtype=dt)

    def run():
        ops.linear(x, w, b, dt, act=ops.ACT_GELU, out=y)

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
    return {"us": round(best * 1e6, 1), "tflops": round(2.0 * M * cout * K / best / 1e12, 1)}


def main():
    names = sys.argv[1:] or list(SHAPES)
    out = {}
    for name in names:
        cin, cout, H, stride, nb, ps = SHAPES[name]
        out[name] = bench(cin, cout, H, stride, nb, ps)
        out[name + "@halfK"] = bench(cin // 2, cout, H, stride, nb, ps)
        out[name + "@dense"] = bench_dense(cin, cout, H, stride, nb)
        print(name, out[name], "half K", out[name + "@halfK"], "dense", out[name + "@dense"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
