"""Which library kernel torch.nn.functional.linear (hipBLASLt) picks for the token-GEMM shapes, and its time:
run under `rocprofv3 --kernel-trace --stats`; the kernel names encode the library's macro tile, depth and
schedule.  Reference only (the product path never calls the library).   usage: python tools/hipblaslt_probe.py"""
import torch

SHAPES = {"enc_fc1": (9280, 3072, 768), "enc_fc2": (9280, 768, 3072), "enc_proj": (9280, 768, 768),
          "dec_fc1": (16448, 2048, 512), "dec_fc2": (16448, 512, 2048), "dec_proj": (16448, 512, 512)}
for name, (M, N, K) in SHAPES.items():
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    for _ in range(10):
        torch.nn.functional.linear(x, w, b)
    torch.cuda.synchronize()
    print(name, flush=True)
