"""Kodak eval harness and score-map producer on the MI355X.

* tmae_image_scores (quadtree + Laplacian + resizes + patch means on the device) is bit-exact with the
  scores the reference's own generate_scores_file glue produced for Kodak (tests/golden/kodak.npz;
  cv2 arithmetic restated, parity with OpenCV itself unpinned), for both image orientations;
* compute_metrics (device PSNR / MS-SSIM) against the pytorch_msssim restatement in float64;
* eval_model over the 24 Kodak images (224^2, K=144, seeded weights: no trained checkpoint exists) with
  the reference's per-image pipeline: compress -> Huffman(ids_restore) -> decompress -> metrics; the bpp
  equals the reference formula on the produced streams, the decoded images equal the eval forward's;
* testing.main (the reference CLI) end to end on PNGs with a saved checkpoint: report.txt JSON.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kodak(golden_dir):
    return np.load(os.path.join(golden_dir, "kodak.npz"))


def test_image_scores_device_bit_exact(tmae, kodak):
    from textmae_amd.scores import image_scores, preprocess_image_scores

    idx = [int(i) for i in kodak["gray_idx"]]
    for i in idx:
        got = image_scores(torch.from_numpy(kodak[f"gray{i}"]).cuda()).cpu().numpy()[0]
        np.testing.assert_array_equal(got, kodak["scores"][i])
    # batched by shape, input order kept
    got = preprocess_image_scores([kodak[f"gray{i}"] for i in idx]).numpy()
    np.testing.assert_array_equal(got, kodak["scores"][idx])


def test_image_scores_synthetic_vs_oracle(tmae):
    """odd sizes (uncovered remainder rows of the int(h/2) split), flat regions, a batch of 3"""
    from oracle import scores_oracle as so
    from textmae_amd.scores import image_scores

    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, (3, 301, 277), dtype=np.uint8)
    imgs[1, :150] = 100                 # flat block: never judged (std 0), splits to the bottom and merges
    imgs[2] = (np.arange(277)[None, :] * 7 % 256).astype(np.uint8)
    got = image_scores(torch.from_numpy(imgs).cuda()).cpu().numpy()
    for b in range(3):
        np.testing.assert_array_equal(got[b], so.image_scores(imgs[b]))


def test_compute_metrics_vs_oracle(tmae):
    from oracle.thirdparty import ms_ssim
    from textmae_amd.testing import compute_metrics

    g = torch.Generator().manual_seed(2)
    org = torch.rand(2, 3, 224, 231, generator=g)
    rec = (org + 0.05 * torch.randn(2, 3, 224, 231, generator=g)).clamp(-0.1, 1.1)
    m = compute_metrics(org.cuda(), rec.cuda())
    qa = (org.double() * 255).clamp(0, 255).round()
    qb = (rec.double() * 255).clamp(0, 255).round()
    ref_psnr = 20 * math.log10(255) - 10 * math.log10(float((qa - qb).pow(2).mean()))
    ref_ms = float(ms_ssim(qa, qb, data_range=255))
    assert abs(m["psnr"] - ref_psnr) < 1e-4
    assert abs(m["ms-ssim"] - ref_ms) < 1e-5


def _model(tmae):
    from oracle.mcm_oracle import MCMConfig, make_state_dict

    cfg = MCMConfig(img_size=224, num_keep_patches=144)
    m = tmae.MCM(**cfg.kwargs())
    full = m.state_dict()
    full.update(make_state_dict(cfg, 17))
    m.load_state_dict(full)
    m = m.cuda().eval()
    m.update(force=True)
    return m


def test_kodak_eval_report(tmae, kodak):
    from oracle.thirdparty import ms_ssim
    from textmae_amd.huffman import HuffmanCoding
    from textmae_amd.testing import bits_per_pixel, eval_model, inference

    m = _model(tmae)
    imgs = [(torch.from_numpy(kodak["rgb224"][i].astype(np.float32) / 255.0).permute(2, 0, 1).unsqueeze(0).contiguous(),
             (768, 512)) for i in range(24)]
    scores = torch.from_numpy(kodak["scores"])
    rep = eval_model(m, None, imgs, scores)
    assert set(rep) == {"psnr", "ms-ssim", "bpp", "encoding_time", "decoding_time"}
    assert all(math.isfinite(v) for v in rep.values())
    # per image: the reference formula on the streams, and the metrics of the decoded image
    bpps, psnrs = [], []
    for i in (0, 5, 23):
        x = imgs[i][0].cuda()
        s = scores[i:i + 1].cuda()
        enc = m.compress(x, s)
        bits, shape, dev = HuffmanCoding().compress(enc["ids_restore"])
        assert len(bits) == 1508
        dec = m.decompress(enc["string"], enc["shape"], enc["ids_restore"])
        with torch.no_grad():
            fwd = m(x, s)
        assert torch.equal(dec["x_hat"], fwd["x_hat"])
        rv = inference(m, imgs[i][0], imgs[i][1], scores[i:i + 1])
        assert rv["bpp"] == pytest.approx(bits_per_pixel(enc["string"], bits, 224 * 224), rel=0, abs=0)
        qa = (x.double().cpu() * 255).clamp(0, 255).round()
        qb = (dec["x_hat"].double().cpu() * 255).clamp(0, 255).round()
        ref_psnr = 20 * math.log10(255) - 10 * math.log10(float((qa - qb).pow(2).mean()))
        assert abs(rv["psnr"] - ref_psnr) < 1e-4
        assert abs(rv["ms-ssim"] - float(ms_ssim(qa, qb, data_range=255))) < 1e-5
        bpps.append(rv["bpp"])
        psnrs.append(rv["psnr"])
    print(f"Kodak-24 (seeded weights): {json.dumps(rep)}")


def test_testing_main_cli(tmae, kodak, tmp_path):
    """the reference CLI (testing.py:168-250) on 3 PNGs: checkpoint -> update(force=True) -> report.txt;
    no <dataset>_scores/test.pt, so the device score producer supplies total_scores"""
    from PIL import Image

    from textmae_amd import testing

    ds = tmp_path / "kodak3"
    ds.mkdir()
    for i in range(3):
        Image.fromarray(kodak["rgb224"][i]).save(ds / f"kodim{i + 1:02d}.png")
    m = _model(tmae)
    ck = tmp_path / "best_model.pth"
    torch.save({"model": {k: v.cpu() for k, v in m.state_dict().items()}}, ck)
    out = tmp_path / "rec"
    rep = testing.main(["-d", str(ds), "-o", str(out), "--cuda", "-c", str(ck), "--num_keep_patches", "144",
                        "--input_size", "224"])
    saved = json.load(open(out / "report.txt"))
    assert saved["name"] == "MCM" and set(saved["results"]) == {"psnr", "ms-ssim", "bpp", "encoding_time",
                                                                 "decoding_time"}
    assert saved["results"]["bpp"] == rep["results"]["bpp"]
    assert len(list(out.glob("*.png"))) == 3
