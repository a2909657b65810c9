"""MaskedAutoencoderViT host side (CPU): seeded construction reproduces the reference weights, the
oracle restatement reproduces the reference's own outputs (tests/golden/mae_forward.npz, made by
running models/MAE/models_mae.py here), and the surface matches (names, factories)."""
import hashlib
import os

import numpy as np
import pytest
import torch

from oracle.mae_oracle import mae_forward


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "mae_forward.npz"))


def sha16(sd):
    a = np.concatenate([v.float().numpy().ravel() for v in sd.values() if v.numel()])
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def test_seeded_init_matches_reference(tmae, golden):
    torch.manual_seed(0)
    m = tmae.mae_vit_base_patch16_dec512d8b()
    assert sha16(m.state_dict()) == str(golden["init_sha_seed0"])
    keys = m.state_dict().keys()  # order is pinned by the hash (values hashed in state_dict order)
    for k in ("cls_token", "pos_embed", "mask_token", "patch_embed.proj.weight", "blocks.11.mlp.fc2.bias",
              "decoder_blocks.7.attn.qkv.weight", "decoder_pred.weight", "norm.weight", "decoder_norm.bias"):
        assert k in keys


def test_oracle_vs_reference_config1(tmae, golden):
    torch.manual_seed(0)
    sd = tmae.mae_vit_base_patch16_dec512d8b().state_dict()
    imgs = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    noise = torch.from_numpy(golden["noise"])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    with torch.no_grad():
        loss, pred, mask = mae_forward(sd, imgs, noise, 0.75, 16, 12, 16, 12, 8)
    np.testing.assert_array_equal(mask.numpy(), golden["mask"])
    np.testing.assert_allclose(float(loss), float(golden["loss"]), rtol=1e-5)
    np.testing.assert_allclose(pred[:, ::7].numpy(), golden["pred_rows"], rtol=1e-4, atol=1e-5)


def test_oracle_vs_reference_tiny_norm_pix(golden):
    sd = {k[len("tiny_sd."):]: torch.from_numpy(golden[k]) for k in golden.files if k.startswith("tiny_sd.")}
    loss, pred, mask = mae_forward(sd, torch.from_numpy(golden["tiny_imgs"]), torch.from_numpy(golden["tiny_noise"]),
                                   0.6, 16, 2, 1, 2, 1, norm_pix=True)
    np.testing.assert_array_equal(mask.numpy(), golden["tiny_mask"])
    np.testing.assert_allclose(float(loss), float(golden["tiny_loss"]), rtol=1e-5)
    np.testing.assert_allclose(pred.numpy(), golden["tiny_pred"], rtol=1e-4, atol=1e-5)


def test_factories_and_forward_guards(tmae):
    m = tmae.mae_vit_large_patch16_dec512d8b()
    assert m.pos_embed.shape == (1, 197, 1024) and len(m.blocks) == 24 and m.decoder_pred.out_features == 768
    h = tmae.mae_vit_huge_patch14_dec512d8b()
    assert h.patch_embed.patch_size == (14, 14) and h.blocks[0].attn.num_heads == 16
    with pytest.raises(ValueError, match="GPU"):
        m(torch.zeros(1, 3, 224, 224))
    x = torch.arange(2 * 196 * 3, dtype=torch.float32).reshape(2, 196, 3)
    assert m.patchify(m.unpatchify(torch.randn(2, 196, 768))).shape == (2, 196, 768)
    assert x.shape == (2, 196, 3)
