"""Kodak eval harness and score-map producer, host side (no GPU): the HuffmanCoding drop-in (host C++ behind
the C ABI) against the reference's own strings and code tables (tests/golden/huffman.npz, made by
tools/gen_golden_eval.py from utils/huffman.py), the reference bpp formula, and the score-map oracle
against the scores the reference's generate_scores_file / utils/map.py / utils/distribution.py produced
for Kodak (tests/golden/kodak.npz; cv2 calls restated, see oracle/scores_oracle.py)."""
import os

import numpy as np
import pytest
import torch


@pytest.fixture(scope="module")
def huff(golden_dir):
    return np.load(os.path.join(golden_dir, "huffman.npz"))


def _names(huff):
    return [str(n) for n in huff["names"]]


def test_huffman_matches_reference_bits_and_codes(tmae, huff):
    from textmae_amd.huffman import HuffmanCoding

    for name in _names(huff):
        vals = torch.from_numpy(huff[f"{name}_values"])
        h = HuffmanCoding()
        bits, shape, dev = h.compress(vals)
        ref_bits = "".join(chr(48 + int(b)) for b in huff[f"{name}_bits"])
        assert bits == ref_bits, name
        assert shape == vals.shape
        # code table: same symbols in the same (pre-order) order with the same codes
        syms = huff[f"{name}_syms"]
        assert list(h.codes.keys()) == [int(s) for s in syms], name
        codes = "".join(h.codes[int(s)] for s in syms)
        assert codes == "".join(chr(48 + int(b)) for b in huff[f"{name}_codes"])
        assert h.reverse_mapping == {v: k for k, v in h.codes.items()}
        back = h.decompress(bits, shape, dev)
        assert torch.equal(back, vals), name


def test_huffman_ids_restore_bit_count(tmae):
    """a permutation of L = 196 has equal frequencies: 60 codes of 7 bits and 136 of 8 (1508 bits), as the
    side info of every Kodak image at K=144 of 224^2 (testing.py:71-74, 88-89)"""
    from textmae_amd.huffman import HuffmanCoding

    ids = torch.argsort(torch.rand(1, 196, generator=torch.Generator().manual_seed(3)), 1)
    bits, _, _ = HuffmanCoding().compress(ids)
    assert len(bits) == 1508


def test_huffman_single_symbol_like_reference(tmae):
    """one distinct value gets the empty code: encode gives '' and decompress fails on the view, as the
    reference's does (huffman.py:99-103, 133-139, 170)"""
    from textmae_amd.huffman import HuffmanCoding

    h = HuffmanCoding()
    bits, shape, dev = h.compress(torch.full((5,), 7, dtype=torch.int64))
    assert bits == "" and h.codes == {7: ""}
    with pytest.raises(RuntimeError):
        h.decompress(bits, shape, dev)


def test_bits_per_pixel_counts_first_z_string_only(tmae):
    from textmae_amd.testing import bits_per_pixel

    strings = [[b"y" * 100], [b"z" * 7, b"z" * 9]]
    assert bits_per_pixel(strings, "0" * 1508, 224 * 224) == pytest.approx((107 * 8 + 1508) / (224 * 224))


def test_score_oracle_reproduces_reference_scores(golden_dir):
    from oracle import scores_oracle as so

    k = np.load(os.path.join(golden_dir, "kodak.npz"))
    for i in k["gray_idx"]:
        got = so.image_scores(k[f"gray{int(i)}"])
        np.testing.assert_array_equal(got, k["scores"][int(i)])


def test_resize_linear_identity_and_constant():
    from oracle import scores_oracle as so

    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    assert np.array_equal(so.resize_linear(a, 53, 37), a)          # same size: identity
    c = np.full((120, 90), 77, dtype=np.uint8)
    assert (so.resize_linear(c, 224, 224) == 77).all()              # constant stays constant


def test_ms_ssim_oracle_identity():
    from oracle.thirdparty import ms_ssim

    x = torch.rand(1, 3, 224, 224, generator=torch.Generator().manual_seed(1)) * 255
    assert float(ms_ssim(x, x, data_range=255)) == pytest.approx(1.0, abs=1e-6)


def test_load_checkpoint_reference_save_model_layout(tmae, tmp_path):
    """testing.load_checkpoint reads what the reference's save_model writes (model_utils.py:30-55):
    {'model', 'optimizer', 'aux_optimizer', 'epoch', 'scaler', 'args': argparse.Namespace}, weights-only"""
    import argparse

    import torch

    from textmae_amd import testing

    kw = dict(encoder_embed_dim=64, encoder_depth=1, encoder_num_heads=2, decoder_embed_dim=32, decoder_depth=1,
              decoder_num_heads=2, latent_depth=48, hyperprior_depth=24)
    torch.manual_seed(0)
    m = tmae.MCM(img_size=64, num_keep_patches=16, **kw)
    opt = torch.optim.Adam([p for n, p in m.named_parameters() if not n.endswith(".quantiles")], lr=1e-4)
    aux = torch.optim.Adam([p for n, p in m.named_parameters() if n.endswith(".quantiles")], lr=1e-4)
    ck = {"model": m.state_dict(), "optimizer": opt.state_dict(), "aux_optimizer": aux.state_dict(), "epoch": 3,
          "scaler": {"scale": 65536.0, "growth_factor": 2.0}, "args": argparse.Namespace(lr=1e-4, batch_size=8)}
    path = tmp_path / "best_model.pth"
    torch.save(ck, path)
    net = testing.load_checkpoint(16, str(path), img_size=64, **kw)
    got = net.state_dict()
    for k, v in m.state_dict().items():
        assert torch.equal(got[k], v), k
