"""One eager MCM training step at the bench configuration (ViT-B, 256^2, K=144, bf16, seeded weights, inputs and
noise) with its gradients saved to a file, so that two library builds (TMAE_LIB=...) can be compared bit for bit:
    python tools/train_dump.py out_a.pt [batch];  TMAE_LIB=ab/lib....so python tools/train_dump.py out_b.pt
    python tools/train_dump.py --compare out_a.pt out_b.pt"""
import sys

import torch

sys.path.insert(0, ".")


def main():
    if sys.argv[1] == "--compare":
        a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        print(f"{len(a)} gradients, {len(a) - len(bad)} bitwise equal")
        for k in bad[:20]:
            print(k, f"DIFFERS max {float((a[k] - b[k]).abs().max()):.3e}")
        sys.exit(1 if bad else 0)
    import bench
    import textmae_amd
    from textmae_amd import engine
    from textmae_amd.optim import configure_optimizers
    from textmae_amd.rd_loss import RateDistortionLoss

    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    torch.manual_seed(0)
    m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
    m.compute_dtype = torch.bfloat16
    m.distortion = "ssim+l1"
    opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
    crit = RateDistortionLoss(lmbda=1e-2)
    imgs, scores = bench.synthetic_inputs(B, 256, m.encoder_embed.num_patches, 2000, "cuda")
    torch.manual_seed(1)
    torch.cuda.manual_seed(1)
    engine.train_step(m, crit, imgs, scores, opt, aux, clip_max_norm=1.0)
    torch.cuda.synchronize()
    # the parameters after one clipped Adam step carry every gradient
    torch.save({k: v.detach().float().cpu() for k, v in m.named_parameters()}, sys.argv[1])
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
