"""Whole eager MCM forwards and nothing else (bench.py's config-2 model and inputs: ViT-B, 256^2, K=144, batch 64,
bf16, eval, distortion "none"), for PMC passes whose per-forward numbers must not mix in other work: every
dispatch from the first forward's ids_shuffle on belongs to a forward (tools/pmc_family.py counts from there).
    python tools/fwd_only.py [forwards] [batch]"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().eval()
m.compute_dtype = torch.bfloat16
m.distortion = "none"
imgs, scores = bench.synthetic_inputs(B, 256, m.encoder_embed.num_patches, 1000, "cuda")
with torch.no_grad():
    for _ in range(n):
        m(imgs, scores)
torch.cuda.synchronize()
print(f"{n} forwards done")
