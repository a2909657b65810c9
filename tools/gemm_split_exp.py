"""Does desynchronising workgroups hide the token GEMM's epilogue?  enc fc1 (9280 x 3072 x 768, GELU) as one
launch, as two N-halves back to back, and as two N-halves on two streams at once (optionally the second started
`delay` cycles later), each replayed 20x from a HIP graph.  python tools/gemm_split_exp.py [delay_cycles ...]"""
import json
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import _lib, ops  # noqa: E402


def lin(x, w, b, out, n0, N, ldo, act=1):
    M, K = x.shape
    _lib.call("tmae_linear_fwd", x.data_ptr(), 0, K, M, 0, 0, w[n0:].data_ptr(), b[n0:].data_ptr(),
              out.data_ptr() + 2 * n0, 0, ldo, None, 0, M, N, K, act, ops.TMAE_BF16, torch.cuda.current_stream().cuda_stream)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    with torch.cuda.stream(s0):
        fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return round(best, 1)


def main():
    delays = [int(v) for v in sys.argv[1:]] or [0, 20000, 40000]
    M, N, K = 9280, 3072, 768
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    res = {"one": timed(lambda: lin(x, w, b, y, 0, N, N))}
    res["halves_serial"] = timed(lambda: (lin(x, w, b, y, 0, N // 2, N), lin(x, w, b, y, N // 2, N // 2, N)))

    def conc(delay):
        def f():
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            lin(x, w, b, y, 0, N // 2, N)
            with torch.cuda.stream(side):
                if delay:
                    torch.cuda._sleep(delay)
                lin(x, w, b, y, N // 2, N // 2, N)
            main.wait_stream(side)
        return f
    for d in delays:
        res[f"halves_concurrent_delay{d}"] = timed(conc(d))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
