"""One eval MCM forward at the bench configuration (ViT-B, 256^2, K=144, bf16, seeded weights and inputs) saved to a
file, so that two library builds (TMAE_LIB=...) can be compared bit for bit:
    python tools/fwd_dump.py out_a.pt [batch];  TMAE_LIB=ab/lib....so python tools/fwd_dump.py out_b.pt
    python tools/fwd_dump.py --compare out_a.pt out_b.pt"""
import sys

import torch

sys.path.insert(0, ".")


def main():
    if sys.argv[1] == "--compare":
        a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        for k in a:
            print(k, "bitwise equal" if k not in bad else f"DIFFERS max {float((a[k] - b[k]).abs().max()):.3e}")
        sys.exit(1 if bad else 0)
    import bench
    import textmae_amd

    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    torch.manual_seed(0)
    m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().eval()
    m.compute_dtype = torch.bfloat16
    m.distortion = "none"
    imgs, scores = bench.synthetic_inputs(B, 256, m.encoder_embed.num_patches, 1000, "cuda")
    with torch.no_grad():
        out = m(imgs, scores)
    torch.cuda.synchronize()
    torch.save({"x_hat": out["x_hat"].cpu(), "y": out["likelihoods"]["y"].cpu(), "z": out["likelihoods"]["z"].cpu()},
               sys.argv[1])
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
