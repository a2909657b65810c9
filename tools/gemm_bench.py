"""Micro-benchmark of the MFMA GEMM on the hot path's token-GEMM shapes, beside torch.matmul
(hipBLASLt) on the same shapes as an achievable-speed reference.  Interleaved rounds, one process.
Forced tiles: a variant library (tools/build_variant.sh <name> gemm.hip -DTMAE_GEMM_TILE=<index>, TMAE_LIB=...)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402
from textmae_amd import ops  # noqa: E402

SHAPES = {  # name: (M, N, K, act)
    "enc_qkv": (9280, 2304, 768, 0), "enc_fc1": (9280, 3072, 768, 1), "enc_fc2": (9280, 768, 3072, 0),
    "enc_proj": (9280, 768, 768, 0), "dec_qkv": (16448, 1536, 512, 0), "dec_fc1": (16448, 2048, 512, 1),
    "dec_fc2": (16448, 512, 2048, 0), "big": (8192, 8192, 8192, 0), "enc_fc1_noact": (9280, 3072, 768, 0), "dec_proj": (16448, 512, 512, 0),
}


def ev_time(fn, reps):
    """GPU time per call: reps calls captured in one HIP graph, replayed (not the host's launch rate)"""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    dt = torch.bfloat16
    out = {}
    torch.manual_seed(0)
    args = sys.argv[1:]
    eager = 0  # --eager N: N plain launches of each GEMM, no graphs or timing (PMC passes: tools/gemm_pmc.sh)
    if args and args[0] == "--eager":
        eager, args = int(args[1]), args[2:]
    names = args or list(SHAPES)
    for name in names:
        M, N, K, act = SHAPES[name]
        x = torch.randn(M, K, device="cuda").to(dt)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=dt)
        mine = lambda: ops.linear(x, w, b, dt, act=act, out=y)
        ref = lambda: torch.nn.functional.linear(x, w, b.to(dt))
        if eager:
            for _ in range(eager):
                mine()
                ref()
            torch.cuda.synchronize()
            print(name, "eager", eager, flush=True)
            continue
        reps = 20 if name != "big" else 5
        fl = 2.0 * M * N * K
        res = {}
        tm = [ev_time(mine, reps) for _ in range(5)]
        res["us"] = round(min(tm) * 1e6, 1)
        res["tf"] = round(fl / min(tm) / 1e12, 1)
        tr = [ev_time(ref, reps) for _ in range(5)]
        res["torch_tf"] = round(fl / min(tr) / 1e12, 1)
        mine()
        # bit pattern checksum: equal across variant libraries that keep the MFMA k-order
        res["bits"] = int(y.view(torch.int16).to(torch.int64).mul_(torch.arange(1, N + 1, device="cuda")).sum().item())
        out[name] = res
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
