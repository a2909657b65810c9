"""Micro-benchmark of the LIC 3x3 convs at the bench shapes (batch 64, 12x12 latent grid, bf16): the
serial slice-stack layers (2 problems: mean + scale) and h_a's first layer, on the halo-staged kernel.
Prints us per launch and
TFLOP/s.  Under rocprofv3 --pmc each launch is one dispatch of the listed shape."""
import json
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops  # noqa: E402

SHAPES = {  # name: (cin, cout, problems)
    "ms_224_176": (224, 176, 2), "ms_176_128": (176, 128, 2), "ms_128_80": (128, 80, 2), "ms_80_32": (80, 32, 2),
    "first_96_224": (96, 224, 2), "ha_384_384": (384, 384, 1),
}


def main():
    names = sys.argv[1:] or list(SHAPES)
    B, H, dt = 64, 12, torch.bfloat16
    out = {}
    for name in names:
        cin, cout, nb = SHAPES[name]
        x = torch.randn(B * H * H, cin, device="cuda").to(dt)
        w = (torch.randn(nb, cout, 9 * cin, device="cuda") / (9 * cin) ** 0.5).to(dt)
        b = torch.randn(nb, cout, device="cuda")
        y = torch.empty(nb, B * H * H, cout, device="cuda", dtype=dt)
        strides = {"w": (0, cout * 9 * cin), "b": (0, cout), "y": (0, B * H * H * cout)}

        def run():
            ops.conv3x3(x, cin, cin, B, H, H, w, b, y, cout, cout, dt, act=ops.ACT_GELU, nb=(1, nb), strides=strides)

        run()
        # 20 launches captured in one HIP graph and replayed: GPU time, not the host's launch rate
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
        fl = 2.0 * nb * B * H * H * cout * 9 * cin
        out[name] = {"us": round(best * 1e6, 1), "tflops": round(fl / best / 1e12, 1)}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
