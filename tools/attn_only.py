"""Decoder / encoder attention forward alone at the bench shapes (batch 64), for PMC passes:
python tools/attn_only.py [dec|enc] [reps]"""
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "dec"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, T, H, dh = (64, 257, 16, 32) if which == "dec" else (64, 145, 12, 64)
D = H * dh
qkv = torch.randn(B * T, 3 * D, device="cuda").to(torch.bfloat16)
o = torch.empty(B * T, D, device="cuda", dtype=torch.bfloat16)
for _ in range(reps):
    ops.mha(qkv, B, T, H, dh, dh ** -0.5, torch.bfloat16, out=o)
torch.cuda.synchronize()
