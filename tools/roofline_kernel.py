"""Launch bench.py's roofline kernel (encoder fc1 + GELU GEMM, M = 64*145, N = 3072, K = 768, bf16)
`reps` times on its own, for rocprofv3 PMC passes (tools/pmc_traffic.py)."""
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops  # noqa: E402


def main(reps=20):
    M, N, K = 64 * 145, 3072, 768
    dt = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).to(dt)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    b = torch.randn(N, device="cuda", generator=g)
    y = torch.empty(M, N, device="cuda", dtype=dt)
    for _ in range(reps):
        ops.linear(x, w, b, dt, act=ops.ACT_GELU, out=y)
    torch.cuda.synchronize()
    print(ops.gemm_plan(M, N, K, dt), "algorithmic bytes", (M * K + N * K + M * N) * 2 + N * 4)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
