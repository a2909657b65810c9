"""Host-side surface of the drop-in MCM: state_dict / init / constructor parity with the reference.
CPU only (no kernel launches)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch


def test_state_dict_keys_match_reference(golden_dir, tmae):
    ref = json.load(open(os.path.join(golden_dir, "mcm_state_keys.json")))
    m = tmae.MCM(num_keep_patches=144)
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref["keys"].keys())
    for k, shp in ref["keys"].items():
        assert list(sd[k].shape) == shp, k


def test_seeded_init_matches_reference(golden_dir, tmae):
    """torch.manual_seed(0); MCM() gives the reference's initial weights bit for bit"""
    ref = json.load(open(os.path.join(golden_dir, "mcm_state_keys.json")))
    torch.manual_seed(0)
    sd = tmae.MCM(num_keep_patches=144).state_dict()
    sha = hashlib.sha256(np.concatenate([v.float().numpy().ravel() for v in sd.values() if v.numel()]).tobytes())
    assert sha.hexdigest()[:16] == ref["init_sha_seed0"]


def test_quantiles_split_for_aux_optimizer(tmae):
    m = tmae.MCM(num_keep_patches=144)
    aux = [n for n, p in m.named_parameters() if n.endswith(".quantiles") and p.requires_grad]
    assert aux == ["entropy_bottleneck.quantiles"]
    frozen = [n for n, p in m.named_parameters() if not p.requires_grad]
    assert sorted(frozen) == ["decoder_pos_embed", "encoder_pos_embed"]


def test_from_state_dict_roundtrip(tmae):
    torch.manual_seed(1)
    a = tmae.MCM(num_keep_patches=144)
    b = tmae.MCM.from_state_dict(144, a.state_dict())
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_forward_requires_device(tmae):
    m = tmae.MCM(img_size=64, encoder_embed_dim=64, encoder_depth=1, encoder_num_heads=2, decoder_embed_dim=32,
                 decoder_depth=1, decoder_num_heads=1, latent_depth=64, hyperprior_depth=32, num_slices=4,
                 num_keep_patches=16)
    with pytest.raises(ValueError, match="GPU"):
        m(torch.zeros(1, 3, 64, 64), torch.zeros(1, 16))


def test_patchify_roundtrip(tmae):
    m = tmae.MCM(img_size=64, num_keep_patches=16, encoder_depth=0, decoder_depth=0)
    x = torch.randn(2, 3, 64, 64)
    assert torch.equal(m.unpatchify(m.patchify(x)), x)
