"""MaskedAutoencoderViT on the GPU (reference models/MAE/models_mae.py) against the reference's own
outputs (tests/golden/mae_forward.npz, mae_masking.npz) and the pinned oracle (oracle/mae_oracle.py).

Masks and ids are bit-exact; pred / loss in f32 meet max|a-b| / max|b| <= 1e-3 (north_star tolerance);
the bf16 path is bounded separately."""
import os

import numpy as np
import pytest
import torch
from parity_log import check  # noqa: E402

from oracle.mae_oracle import mae_forward

pytestmark = pytest.mark.gpu
DEV = "cuda"


def maxrel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max())


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "mae_forward.npz"))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_masking_bit_exact(tmae, golden_dir, seed):
    f = np.load(os.path.join(golden_dir, "mae_masking.npz"))
    torch.manual_seed(seed)
    noise = torch.rand(4, 196)  # what random_masking drew on the CPU after manual_seed(seed)
    from textmae_amd import ops

    shuf, rest, mask = ops.mae_masking(noise.to(DEV), 49)
    np.testing.assert_array_equal(rest.cpu().numpy(), f[f"s{seed}_ids_restore"])
    np.testing.assert_array_equal(mask.cpu().numpy(), f[f"s{seed}_mask"])
    # the golden gathered x = arange(4 * 196): x_masked = 196 b + kept index
    kept = shuf[:, :49].cpu().numpy() + 196 * np.arange(4)[:, None]
    np.testing.assert_array_equal(kept, f[f"s{seed}_x_masked"][..., 0].astype(np.int64))


def config1(tmae, dtype):
    torch.manual_seed(0)
    m = tmae.mae_vit_base_patch16_dec512d8b()
    m.compute_dtype = dtype
    imgs = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    return m.to(DEV), imgs


def test_config1_f32_vs_reference(tmae, golden):
    m, imgs = config1(tmae, torch.float32)
    with torch.no_grad():
        loss, pred, mask = m(imgs.to(DEV), 0.75, noise=torch.from_numpy(golden["noise"]).to(DEV))
    np.testing.assert_array_equal(mask.cpu().numpy(), golden["mask"])
    check("maxrel:pred_7", maxrel(pred[:, ::7], golden["pred_rows"]), 1e-3)
    np.testing.assert_allclose(pred.double().sum((1, 2)).cpu().numpy(), golden["pred_sum"],
                               rtol=1e-3, atol=1e-3 * float(np.abs(golden["pred_rows"]).max()) * pred[0].numel() ** 0.5)
    np.testing.assert_allclose(float(loss), float(golden["loss"]), rtol=1e-3)


def test_config1_bf16_bounded(tmae, golden):
    m, imgs = config1(tmae, torch.bfloat16)
    with torch.no_grad():
        loss, pred, mask = m(imgs.to(DEV), 0.75, noise=torch.from_numpy(golden["noise"]).to(DEV))
    np.testing.assert_array_equal(mask.cpu().numpy(), golden["mask"])
    ref = torch.from_numpy(golden["pred_rows"]).double()
    l2 = float((pred[:, ::7].double().cpu() - ref).norm() / ref.norm())
    assert l2 < 3e-2, l2
    np.testing.assert_allclose(float(loss), float(golden["loss"]), rtol=3e-2)


def test_tiny_norm_pix_vs_reference(tmae, golden):
    from functools import partial

    m = tmae.MaskedAutoencoderViT(img_size=64, patch_size=16, in_chans=3, embed_dim=64, depth=2, num_heads=2,
                                  decoder_embed_dim=32, decoder_depth=1, decoder_num_heads=1, mlp_ratio=4.0,
                                  norm_layer=partial(torch.nn.LayerNorm, eps=1e-6), norm_pix_loss=True)
    m.load_state_dict({k[len("tiny_sd."):]: torch.from_numpy(golden[k]) for k in golden.files
                       if k.startswith("tiny_sd.")})
    m = m.to(DEV)
    with torch.no_grad():
        loss, pred, mask = m(torch.from_numpy(golden["tiny_imgs"]).to(DEV), 0.6,
                             noise=torch.from_numpy(golden["tiny_noise"]).to(DEV))
    np.testing.assert_array_equal(mask.cpu().numpy(), golden["tiny_mask"])
    check("maxrel:pred", maxrel(pred, golden["tiny_pred"]), 1e-3)
    np.testing.assert_allclose(float(loss), float(golden["tiny_loss"]), rtol=1e-3)


def test_vitl_vs_oracle_and_split_api(tmae):
    """ViT-L encoder (24 x 1024, 16 heads): oracle comparison; forward_encoder -> forward_decoder ->
    forward_loss composes to forward"""
    torch.manual_seed(3)
    m = tmae.mae_vit_large_patch16_dec512d8b().to(DEV)
    imgs = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(4))
    noise = torch.rand(2, 196, generator=torch.Generator().manual_seed(5))
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    with torch.no_grad():
        rl, rp, rm = mae_forward(sd, imgs, noise, 0.75, 16, 16, 16, 24, 8)
        loss, pred, mask = m(imgs.to(DEV), 0.75, noise=noise.to(DEV))
        assert torch.equal(mask.cpu(), rm)
        check("maxrel:pred", maxrel(pred, rp), 1e-3)
        np.testing.assert_allclose(float(loss), float(rl), rtol=1e-3)
        lat, mask2, rest = m.forward_encoder(imgs.to(DEV), 0.75, noise=noise.to(DEV))
        assert lat.shape == (2, 50, 1024) and lat.dtype == torch.float32 and torch.equal(mask2, mask)
        pred2 = m.forward_decoder(lat, rest)
        check("maxrel:pred2", maxrel(pred2, pred), 1e-5)
        np.testing.assert_allclose(float(m.forward_loss(imgs.to(DEV), pred2, mask2)), float(loss), rtol=1e-5)
    # under autograd the parts run the training executor (test_gpu_mae_train.py checks their gradients)
    lat3, mask3, _ = m.forward_encoder(imgs.to(DEV), 0.75, noise=noise.to(DEV))
    assert lat3.requires_grad and torch.equal(mask3, mask)
    check("maxrel:lat_autograd", maxrel(lat3.detach(), lat), 1e-5)


def test_vitl_literal_config4_batch128_bf16_graph(tmae):
    """BASELINE config 4 as written: mae_vit_large_patch16_dec512d8b (models_mae.py:231-236), batch 128, bf16,
    forward replayed as a HIP graph (bench.py --mae-large).  Masks are bit-exact for every image; images 0, 64
    and 127 against the f32 oracle within the bf16 bound (relative L2 of pred); the graph replay equals the
    eager forward bitwise."""
    torch.manual_seed(11)
    m = tmae.mae_vit_large_patch16_dec512d8b().to(DEV).eval()
    m.compute_dtype = torch.bfloat16
    imgs = torch.randn(128, 3, 224, 224, generator=torch.Generator().manual_seed(12))
    noise = torch.rand(128, 196, generator=torch.Generator().manual_seed(13))
    x, nz = imgs.to(DEV), noise.to(DEV)
    with torch.no_grad():
        eager = m(x, 0.75, noise=nz)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(x, 0.75, noise=nz)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = m(x, 0.75, noise=nz)
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out[1], eager[1]) and torch.equal(out[2], eager[2])
    pick = [0, 64, 127]
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    with torch.no_grad():
        rl, rp, rm = mae_forward(sd, imgs[pick], noise[pick], 0.75, 16, 16, 16, 24, 8)
    assert torch.equal(out[2][pick].cpu(), rm)
    pr = out[1][pick].double().cpu()
    per = [float((pr[i] - rp[i].double()).norm() / rp[i].double().norm()) for i in range(3)]
    check("pred_relL2_max_bf16_mae_large_b128", max(per), 1.5e-2)


def test_huge_patch14_vs_oracle(tmae):
    """ViT-H factory (models_mae.py:239-244): patch 14 (588-value patch rows, per-value gather), 32 x 1280,
    16 heads of dim 80 (attention tiles padded to 96), dec512d8b; f32 against the oracle at batch 1"""
    torch.manual_seed(6)
    m = tmae.mae_vit_huge_patch14_dec512d8b().to(DEV)
    imgs = torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(7))
    noise = torch.rand(1, 256, generator=torch.Generator().manual_seed(8))
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    with torch.no_grad():
        rl, rp, rm = mae_forward(sd, imgs, noise, 0.75, 14, 16, 16, 32, 8)
        loss, pred, mask = m(imgs.to(DEV), 0.75, noise=noise.to(DEV))
    assert pred.shape == (1, 256, 588) and torch.equal(mask.cpu(), rm)
    check("maxrel:pred", maxrel(pred, rp), 1e-3)
    np.testing.assert_allclose(float(loss), float(rl), rtol=1e-3)


def test_head_dim_reports(tmae):
    from functools import partial

    m = tmae.MaskedAutoencoderViT(img_size=32, patch_size=16, embed_dim=96, depth=1, num_heads=2,
                                  decoder_embed_dim=32, decoder_depth=1, decoder_num_heads=1,
                                  norm_layer=partial(torch.nn.LayerNorm, eps=1e-6)).to(DEV)
    with torch.no_grad(), pytest.raises(ValueError, match="head dim 48"):
        m(torch.zeros(1, 3, 32, 32, device=DEV))
