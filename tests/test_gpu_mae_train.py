"""MaskedAutoencoderViT training path (mae_train.py) against autograd through the pinned f32 oracle
(oracle/mae_oracle.py, the reference models_mae.py forward restated; pinned to the reference's own outputs by
tests/golden/mae_forward.npz in test_gpu_mae.py).

loss and pred in f32 meet max|a-b| / max|b| <= 1e-3 (north_star tolerance), every parameter gradient
max|a-b| / max|b| <= 1e-3 (measured ~1e-6); the bf16 path is bounded by the relative L2 of each gradient."""
import os
from functools import partial

import pytest
import torch
from parity_log import check  # noqa: E402

from oracle.mae_oracle import mae_decoder, mae_encoder, mae_forward

pytestmark = pytest.mark.gpu
DEV = "cuda"


def maxrel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def oracle_grads(m, imgs, noise, ratio, patch, heads, dec_heads, depth, dec_depth, norm_pix):
    sd = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    loss, pred, mask = mae_forward(sd, imgs, noise, ratio, patch, heads, dec_heads, depth, dec_depth,
                                   norm_pix=norm_pix)
    loss.backward()
    return loss.detach(), pred.detach(), mask, {k: v.grad for k, v in sd.items()}


def run_train(m, imgs, noise, ratio):
    m.zero_grad(set_to_none=True)
    loss, pred, mask = m(imgs.to(DEV), ratio, noise=noise.to(DEV))
    loss.backward()
    for n, p in m.named_parameters():
        if not p.requires_grad:
            assert p.grad is None, n  # pos_embed / decoder_pos_embed: fixed sin-cos tables
    return loss.detach(), pred.detach(), mask, {n: p.grad for n, p in m.named_parameters() if p.requires_grad}


def tiny(tmae, norm_pix, dec_dim=32, patch=16):
    torch.manual_seed(21)
    return tmae.MaskedAutoencoderViT(img_size=4 * patch, patch_size=patch, in_chans=3, embed_dim=64, depth=2, num_heads=2,
                                     decoder_embed_dim=dec_dim, decoder_depth=2, decoder_num_heads=1, mlp_ratio=4.0,
                                     norm_layer=partial(torch.nn.LayerNorm, eps=1e-6), norm_pix_loss=norm_pix).to(DEV)


@pytest.mark.parametrize("norm_pix,patch", [(False, 16), (True, 16), (False, 14), (True, 14)])
def test_tiny_grads_f32_vs_oracle(tmae, norm_pix, patch):
    """patch 14 (588-value patch rows, zero-padded to 592 in the gathered patches, the weight copy and the weight
    gradient) as well as 16"""
    m = tiny(tmae, norm_pix, patch=patch)
    imgs = torch.randn(3, 3, 4 * patch, 4 * patch, generator=torch.Generator().manual_seed(22))
    noise = torch.rand(3, 16, generator=torch.Generator().manual_seed(23))
    rl, rp, rm, rg = oracle_grads(m, imgs, noise, 0.75, patch, 2, 1, 2, 2, norm_pix)
    loss, pred, mask, grads = run_train(m, imgs, noise, 0.75)
    assert torch.equal(mask.cpu(), rm)
    sfx = f"np{int(norm_pix)}" + ("" if patch == 16 else f"_p{patch}")
    check(f"maxrel:mae_train_tiny_pred_{sfx}", maxrel(pred, rp), 1e-3)
    assert abs(float(loss) - float(rl)) <= 1e-3 * abs(float(rl))
    worst = 0.0
    for name, g in grads.items():
        worst = max(worst, maxrel(g, rg[name]))
    check(f"maxrel:mae_train_tiny_grads_{sfx}", worst, 1e-3)


def test_huge_patch14_grads_f32_vs_oracle(tmae):
    """mae_vit_huge_patch14_dec512d8b (models_mae.py:239-244: patch 14, 588-value patch rows; 1280 wide, 16 heads
    of 80, 32 blocks) trains: batch 1, f32, loss / pred / every parameter gradient against autograd through the
    oracle"""
    torch.manual_seed(29)
    m = tmae.mae_vit_huge_patch14_dec512d8b().to(DEV)
    imgs = torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(30))
    noise = torch.rand(1, 256, generator=torch.Generator().manual_seed(31))
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    rl, rp, rm, rg = oracle_grads(m, imgs, noise, 0.75, 14, 16, 16, 32, 8, False)
    loss, pred, mask, grads = run_train(m, imgs, noise, 0.75)
    assert torch.equal(mask.cpu(), rm)
    check("maxrel:mae_train_huge_pred", maxrel(pred, rp), 1e-3)
    assert abs(float(loss) - float(rl)) <= 1e-3 * abs(float(rl))
    worst, name_w = 0.0, None
    for name, g in grads.items():
        r = maxrel(g, rg[name])
        if r > worst:
            worst, name_w = r, name
    check("maxrel:mae_train_huge_grads", worst, 1e-3, note=name_w)


def test_vitb_grads_f32_vs_oracle(tmae):
    """mae_vit_base_patch16_dec512d8b (models_mae.py:223-228) at batch 2: every gradient against the oracle"""
    torch.manual_seed(24)
    m = tmae.mae_vit_base_patch16_dec512d8b().to(DEV)
    imgs = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(25))
    noise = torch.rand(2, 196, generator=torch.Generator().manual_seed(26))
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    rl, rp, rm, rg = oracle_grads(m, imgs, noise, 0.75, 16, 12, 16, 12, 8, False)
    loss, pred, mask, grads = run_train(m, imgs, noise, 0.75)
    assert torch.equal(mask.cpu(), rm)
    check("maxrel:mae_train_vitb_pred", maxrel(pred, rp), 1e-3)
    assert abs(float(loss) - float(rl)) <= 1e-3 * abs(float(rl))
    worst, name_w = 0.0, None
    for name, g in grads.items():
        r = maxrel(g, rg[name])
        if r > worst:
            worst, name_w = r, name
    check("maxrel:mae_train_vitb_grads", worst, 1e-3, note=name_w)


@pytest.mark.parametrize("norm_pix", [False, True])
def test_split_encoder_decoder_grads_f32_vs_oracle(tmae, norm_pix):
    """forward_encoder -> forward_decoder -> forward_loss as separate module calls under autograd (models_mae.py
    150-214, the reference's nn.Module behaviour): one autograd node per part, the HIP backward of each; every
    gradient against autograd through the oracle's whole forward"""
    m = tiny(tmae, norm_pix)
    imgs = torch.randn(3, 3, 64, 64, generator=torch.Generator().manual_seed(40))
    noise = torch.rand(3, 16, generator=torch.Generator().manual_seed(41))
    rl, rp, rm, rg = oracle_grads(m, imgs, noise, 0.75, 16, 2, 1, 2, 2, norm_pix)
    m.zero_grad(set_to_none=True)
    lat, mask, rest = m.forward_encoder(imgs.to(DEV), 0.75, noise=noise.to(DEV))
    pred = m.forward_decoder(lat, rest)
    loss = m.forward_loss(imgs.to(DEV), pred, mask)
    loss.backward()
    assert torch.equal(mask.cpu(), rm)
    check(f"maxrel:mae_split_pred_np{int(norm_pix)}", maxrel(pred.detach(), rp), 1e-3)
    assert abs(float(loss.detach()) - float(rl)) <= 1e-3 * abs(float(rl))
    worst = 0.0
    for n, p_ in m.named_parameters():
        if not p_.requires_grad:
            assert p_.grad is None, n
            continue
        worst = max(worst, maxrel(p_.grad, rg[n]))
    check(f"maxrel:mae_split_grads_np{int(norm_pix)}", worst, 1e-3)


def test_encoder_alone_and_decoder_alone_vs_oracle(tmae):
    """each part alone: forward_encoder under a random projection of the latent (only encoder parameters get
    gradients), forward_decoder of a leaf latent (gradients to the latent and the decoder's parameters only), against
    the oracle's encoder / decoder; a second forward of a part before its backward is refused"""
    m = tiny(tmae, False)
    imgs = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(42))
    noise = torch.rand(2, 16, generator=torch.Generator().manual_seed(43))
    sd = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    enc_names = {n for n, _ in m.named_parameters() if n.startswith(("blocks.", "norm.", "patch_embed.", "cls_token"))}
    # encoder alone
    lat_o, mask_o, rest_o = mae_encoder(sd, imgs, noise, 0.75, 16, 2, 2)
    R = torch.randn(lat_o.shape, generator=torch.Generator().manual_seed(44))
    (lat_o * R).sum().backward()
    m.zero_grad(set_to_none=True)
    lat, mask, rest = m.forward_encoder(imgs.to(DEV), 0.75, noise=noise.to(DEV))
    check("maxrel:mae_enc_alone_latent", maxrel(lat.detach(), lat_o.detach()), 1e-3)
    assert torch.equal(rest.cpu(), rest_o)
    (lat * R.to(DEV)).sum().backward()
    worst = 0.0
    for n, p_ in m.named_parameters():
        if n in enc_names:
            worst = max(worst, maxrel(p_.grad, sd[n].grad))
        else:
            assert p_.grad is None, n
    check("maxrel:mae_enc_alone_grads", worst, 1e-3)
    # decoder alone, on a leaf latent
    for v in sd.values():
        v.grad = None
    x_o = torch.randn(lat_o.shape, generator=torch.Generator().manual_seed(45)).requires_grad_(True)
    pred_o = mae_decoder(sd, x_o, rest_o, 1, 2)
    R2 = torch.randn(pred_o.shape, generator=torch.Generator().manual_seed(46))
    (pred_o * R2).sum().backward()
    m.zero_grad(set_to_none=True)
    x = x_o.detach().to(DEV).requires_grad_(True)
    pred = m.forward_decoder(x, rest_o.to(DEV))
    check("maxrel:mae_dec_alone_pred", maxrel(pred.detach(), pred_o.detach()), 1e-3)
    (pred * R2.to(DEV)).sum().backward()
    check("maxrel:mae_dec_alone_dx", maxrel(x.grad, x_o.grad), 1e-3)
    worst = 0.0
    for n, p_ in m.named_parameters():
        if n in enc_names or not p_.requires_grad:
            assert p_.grad is None, n
        else:
            worst = max(worst, maxrel(p_.grad, sd[n].grad))
    check("maxrel:mae_dec_alone_grads", worst, 1e-3)
    # stale activations
    lat1, _, _ = m.forward_encoder(imgs.to(DEV), 0.75, noise=noise.to(DEV))
    m.forward_encoder(imgs.to(DEV), 0.75, noise=noise.to(DEV))
    with pytest.raises(RuntimeError, match="forward_encoder ran again"):
        lat1.sum().backward()


@pytest.mark.parametrize("patch", [16, 14])
def test_bf16_bounded_and_adam_steps(tmae, patch):
    """bf16 operands: gradients within a relative L2 bound of the f32 oracle; then FusedAdam steps on one batch
    drive the loss down (the training loop a user of the reference runs).  Patch 14: decoder_pred's 588 outputs
    run its weight / data gradients on zero-tailed 592-column copies"""
    from textmae_amd.optim import FusedAdam

    m = tiny(tmae, True, dec_dim=64, patch=patch)
    m.compute_dtype = torch.bfloat16
    imgs = torch.randn(8, 3, 4 * patch, 4 * patch, generator=torch.Generator().manual_seed(27))
    noise = torch.rand(8, 16, generator=torch.Generator().manual_seed(28))
    rl, rp, rm, rg = oracle_grads(m, imgs, noise, 0.75, patch, 2, 1, 2, 2, True)
    loss, pred, mask, grads = run_train(m, imgs, noise, 0.75)
    worst = 0.0
    for name, g in grads.items():
        ref = rg[name].double()
        worst = max(worst, float((g.double().cpu() - ref).norm() / ref.norm().clamp_min(1e-30)))
    check("relL2:mae_train_bf16_grads" + ("" if patch == 16 else f"_p{patch}"), worst, 2e-2)  # measured 9.2e-3
    opt = FusedAdam([p for p in m.parameters() if p.requires_grad], lr=1e-3)
    first = None
    for _ in range(8):
        opt.zero_grad()
        loss, _, _ = m(imgs.to(DEV), 0.75, noise=noise.to(DEV))
        loss.backward()
        opt.step()
        first = float(loss) if first is None else first
    assert float(loss) < 0.9 * first, (first, float(loss))


def test_graphed_mae_step_bitwise(tmae):
    """engine.GraphedMAEStep: replays equal eager steps (loss and weights, bitwise) with injected noise"""
    from textmae_amd.engine import GraphedMAEStep
    from textmae_amd.optim import FusedAdam

    def make():
        m = tiny(tmae, True, dec_dim=64)
        m.compute_dtype = torch.bfloat16
        return m, FusedAdam([p for p in m.parameters() if p.requires_grad], lr=1e-3)

    imgs = [torch.randn(4, 3, 64, 64, generator=torch.Generator().manual_seed(40 + i)).to(DEV) for i in range(4)]
    noise = [torch.rand(4, 16, generator=torch.Generator().manual_seed(50 + i)).to(DEV) for i in range(4)]
    m1, o1 = make()
    eager = []
    for x, nz in zip(imgs, noise):
        o1.zero_grad()
        loss, _, _ = m1(x, 0.75, noise=nz)
        loss.backward()
        o1.step()
        eager.append(float(loss))
    m2, o2 = make()
    step = GraphedMAEStep(m2, o2, imgs[0], 0.75, warmup=1, noise=noise[0])  # the warm-up step is step 0
    graphed = [eager[0]] + [float(step(x, noise=nz)) for x, nz in zip(imgs[1:], noise[1:])]
    assert graphed == eager, (graphed, eager)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), n
