"""tmae_ids_shuffle alone at the bench shape (batch 64, L = 256, K = 144): us per launch from 50 back-to-back launches
timed with events (best of 5); TMAE_LIB selects an A/B library.
    python tools/ids_bench.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import ops  # noqa: E402

res = {}
for name, (B, L, K) in {"bench": (64, 256, 144), "k64": (64, 256, 64), "mae196": (64, 196, 49)}.items():
    g = torch.Generator().manual_seed(5)
    s = torch.rand(B, L, generator=g).cuda()
    ops.ids_shuffle(s, K)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.ids_shuffle(s, K)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 50 * 1e3)
    res[name] = round(best, 2)
print(json.dumps(res))
