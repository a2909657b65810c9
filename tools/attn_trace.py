"""Phase timeline of the one-pass attention backward (mha_bwd1_bf16_kernel) from the TMAE_ATTN_TRACE build
(tools/build_variant.sh attn_trace attention.hip -DTMAE_ATTN_TRACE=1; TMAE_LIB=ab/libtmae_attn_trace.so): one eager
launch per bench shape (encoder T 145 x 12 heads x dh 64, decoder T 257 x 16 x 32, batch 64); wave 0 of every
workgroup stamped s_memtime after the prologue, after every step's barrier, after dK / dV and after dQ.  Prints the
mean cycles of each phase per workgroup.   usage: TMAE_LIB=... python tools/attn_trace.py"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import _lib, train_ops  # noqa: E402


def main():
    lib = _lib.load()
    for name, (B, T, H, dh) in {"enc": (64, 145, 12, 64), "dec": (64, 257, 16, 32)}.items():
        D = H * dh
        torch.manual_seed(0)
        qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
        o = torch.empty(B * T, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * H * T, device="cuda")
        dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
        dqkv = torch.empty_like(qkv)
        train_ops.mha_lse(qkv, B, T, H, dh, dh ** -0.5, torch.bfloat16, o, lse)
        for _ in range(3):
            train_ops.mha_bwd(qkv, o, dout, lse, dqkv, B, T, H, dh, dh ** -0.5, torch.bfloat16)
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 16, dtype=np.uint64)
        lib.tmae_attn_trace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
        tr = buf.reshape(4096, 16).astype(np.int64)[:B * H]
        nw = (T + 31) // 32
        rel = tr - tr[:, :1]
        steps = [int((rel[:, 2 + i] - (rel[:, 1 + i] if i else rel[:, 1])).mean()) for i in range(nw)]
        print(name, {"wgs": B * H, "prologue": int(rel[:, 1].mean()), "steps": steps,
                     "dkdv": int((rel[:, 14] - rel[:, 1 + nw]).mean()), "dq": int((rel[:, 15] - rel[:, 14]).mean()),
                     "total": int(rel[:, 15].mean())}, flush=True)


if __name__ == "__main__":
    main()
