"""Micro-benchmark of the fused slice-transform stack (tmae_lic_stack) at the bench shapes (batch 64,
12x12 latent grid, bf16, mid channels 224/176/128/80/32), alone on the GPU (no side stream):
  ms_<i>:  the mean + scale stacks of serial slice i (2 problems, layer-0 input 32 i y_hat channels)
  lrp_<i>: the lrp stack of slice i (1 problem, 32 (i + 1) channels)
  b_ms / b_lrp: the batched slices 6..11 (12 / 6 problems, 192 / 192 + 32 channels)
Prints us per launch (20 launches replayed from one HIP graph, best of 5) and TFLOP/s.
usage: python tools/lstk_bench.py [name ...]"""
import json
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops  # noqa: E402

MID = [224, 176, 128, 80, 32]
SHAPES = {"ms_0": (0, 0, 2, 1), "ms_3": (96, 0, 2, 1), "ms_5": (160, 0, 2, 1), "lrp_3": (128, 0, 1, 1),
          "lrp_5": (192, 0, 1, 1), "b_ms": (192, 0, 2, 6), "b_lrp": (192, 32, 1, 6)}


def flops(cin0, P, B=64, G=12):
    ch = [cin0] + MID
    return 2.0 * P * B * G * G * 9 * sum(ch[i] * ch[i + 1] for i in range(5))


def main():
    names = sys.argv[1:] or list(SHAPES)
    B, G = 64, 12
    rows = B * G * G
    out = {}
    for name in names:
        c1, c2, nb1, nb2 = SHAPES[name]
        P = nb1 * nb2
        x1 = torch.randn(rows, 384, device="cuda").to(torch.bfloat16)
        chans = [c1 + c2] + MID
        ws = [torch.stack([ops.pack_lic_stack_weight(torch.randn(chans[l + 1], chans[l], 3, 3, device="cuda")
                                                     / (3 * max(chans[l], 1) ** 0.5)) for _ in range(P)])
              for l in range(5)]
        bs = [torch.randn(P, c, device="cuda") * 0.1 for c in MID]
        add = torch.randn(rows, 8064, device="cuda")
        y = torch.empty(P, rows, 32, device="cuda")
        src = torch.randn(rows, 384, device="cuda")
        yb = torch.empty(rows, 384, device="cuda", dtype=torch.bfloat16)
        st = {"a": (224 * nb2, 224), "y": (nb2 * rows * 32, rows * 32), "x2": (0, 32), "src": (0, 32)}
        for l in range(5):
            st[f"w{l}"] = (nb2 * ws[l][0].numel(), ws[l][0].numel())
            st[f"b{l}"] = (nb2 * MID[l], MID[l])
        lrp = name.endswith("lrp") or name.startswith("lrp")

        def run():
            if lrp:
                st["y"] = (0, 32)
                ops.lic_stack(B, G, x1, c1, 384, ws, bs, MID, yb, 384, False, x2=x1 if c2 else None, c2=c2, ld2=384,
                              addend=add, ld_add=8064, lrp_src=src, ld_src=384, nb=(nb1, nb2), strides=st)
            else:
                ops.lic_stack(B, G, x1, c1, 384, ws, bs, MID, y, 32, True, addend=add, ld_add=8064, nb=(nb1, nb2),
                              strides=st)

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
        fl = flops(c1 + c2, P)
        out[name] = {"us": round(best * 1e6, 1), "tflops": round(fl / best / 1e12, 1), "wgs": P * B}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
