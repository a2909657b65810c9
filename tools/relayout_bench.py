"""Time the multi-tensor weight relayout (tmae_relayout_multi) per layout kind on synthetic ViT-B /
LIC-shaped parameters: plain casts (nt), transposes (t, conv_dg) and conv rows (conv)."""
import sys, os, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
import textmae_amd  # noqa: F401
from textmae_amd.mcm_train import _Weights

dev = "cuda"
shapes_lin = [(2304, 768), (768, 768), (3072, 768), (768, 3072)] * 12 + [(1536, 512), (512, 512), (2048, 512), (512, 2048)] * 8
shapes_conv = [(320, 320, 3, 3)] * 16 + [(224, 416, 3, 3)] * 12 + [(128, 224, 3, 3)] * 24 + [(32, 128, 3, 3)] * 24
res = {}
kinds = (("nt", shapes_lin), ("t", shapes_lin), ("conv", shapes_conv), ("conv_dg", shapes_conv))
only = sys.argv[1:]  # e.g. "t": one kind per process, for a per-kind rocprofv3 kernel time
for kind, shapes in kinds:
    if only and kind not in only:
        continue
    W = _Weights(torch.bfloat16)
    ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in shapes]
    for p in ps:
        getattr(W, kind)(p)
    n = sum(p.numel() for p in ps)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for it in range(12):
        with torch.no_grad():
            for p in ps:
                p.add_(0.0)  # new version: every copy is stale
        torch.cuda.synchronize()
        ev[0].record()
        W.refresh()
        ev[1].record()
        torch.cuda.synchronize()
        if it >= 2:
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    ts.sort()
    us = ts[len(ts) // 2]
    res[kind] = {"params": n, "us": round(us, 1), "GB/s": round(n * 6 / us / 1e3, 1)}
    print(kind, res[kind], flush=True)
print(json.dumps(res))
