"""Golden fixtures for the Kodak eval harness and the score-map producer, made from the REAL reference code
(run only in the survey container, where /root/reference exists).

* tests/golden/huffman.npz — the reference's HuffmanCoding (utils/huffman.py, imports cleanly) on
  ids_restore-shaped permutations and on skewed / tie-heavy integer tensors: input values, the bit
  strings and the code tables.
* tests/golden/kodak.npz — the 24 Kodak images (datasets/kodak) resized to 224^2 exactly as the
  reference's test transform does (PIL bicubic, utils/dataloader.py:69-73), as uint8 HWC; the score
  vectors produced by the reference's own generate_scores_file.preprocess_image_scores (with utils/map.py
  and utils/distribution.py) for all 24; and 4 full-resolution grayscale images for the device
  score-map parity test.  cv2 is absent, so a stub module supplies imread / resize / Laplacian /
  convertScaleAbs from oracle/scores_oracle.py (those four calls stay parity-unpinned); everything else
  (quadtree split / merge with numpy float64 statistics, patch means, the product and min-max
  normalisation, the in-place Laplacian-after-merge order) is the reference's code.

    python tools/gen_golden_eval.py
"""
from __future__ import annotations

import glob
import os
import sys
import tempfile
import types

import numpy as np
import torch
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("TMAE_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from oracle import scores_oracle as so  # noqa: E402


def _load(name, path):
    import importlib.util

    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def huffman_golden():
    huff = _load("ref_huffman", os.path.join(REF, "utils", "huffman.py"))
    g = torch.Generator().manual_seed(0)
    cases = {
        "ids_b1_L196": torch.argsort(torch.argsort(torch.rand(1, 196, generator=g), 1), 1),
        "ids_b4_L196": torch.argsort(torch.rand(4, 196, generator=g), 1),
        "ids_b2_L256": torch.argsort(torch.rand(2, 256, generator=g), 1),
        "geometric": torch.from_numpy(np.random.default_rng(1).geometric(0.15, size=(3, 500)).astype(np.int64) - 3),
        "ties": torch.from_numpy(np.random.default_rng(2).integers(0, 6, size=(700,)).astype(np.int64) * 7),
        "two_symbols": torch.tensor([5, 5, 9, 5, 9, 9, 9, 5, 5], dtype=torch.int64),
    }
    out = {}
    for name, t in cases.items():
        h = huff.HuffmanCoding()
        bits, shape, _ = h.compress(t)
        dec = h.decompress(bits, shape, "cpu")
        assert torch.equal(dec, t)
        syms = np.array(list(h.codes.keys()), dtype=np.int64)
        code_str = "".join(h.codes[int(s)] for s in syms)
        out[f"{name}_values"] = t.numpy()
        out[f"{name}_bits"] = np.frombuffer(bits.encode(), dtype=np.uint8) - ord("0")
        out[f"{name}_syms"] = syms
        out[f"{name}_lens"] = np.array([len(h.codes[int(s)]) for s in syms], dtype=np.int32)
        out[f"{name}_codes"] = np.frombuffer(code_str.encode(), dtype=np.uint8) - ord("0")
    np.savez_compressed(os.path.join(OUT, "huffman.npz"), names=np.array(list(cases)), **out)
    print("huffman:", {k: len(out[f"{k}_bits"]) for k in cases})


def kodak_golden():
    files = sorted(glob.glob(os.path.join(REF, "datasets", "kodak", "*.png")))
    assert len(files) == 24
    grays = {os.path.abspath(f): so.rgb_to_gray(np.array(Image.open(f).convert("RGB"))) for f in files}

    def imread(path, flag=None):
        return grays[os.path.abspath(str(path))].copy()

    def resize(img, shape):
        return so.resize_linear(np.asarray(img), shape[0], shape[1])

    def laplacian(img, ddepth, ksize=1):
        assert ksize == 3
        return so.laplacian_abs(img).astype(np.int16)  # |.| folded here; convertScaleAbs below is then identity

    cv2 = types.ModuleType("cv2")
    cv2.IMREAD_GRAYSCALE, cv2.CV_16S = 0, 3
    cv2.imread, cv2.resize, cv2.Laplacian = imread, resize, laplacian
    cv2.convertScaleAbs = lambda x: np.minimum(np.abs(np.asarray(x, dtype=np.int64)), 255).astype(np.uint8)
    sys.modules["cv2"] = cv2
    sys.path.insert(0, REF)
    gsf = _load("ref_generate_scores_file", os.path.join(REF, "generate_scores_file.py"))
    with tempfile.TemporaryDirectory() as td:
        out_file = os.path.join(td, "test.pt")
        gsf.preprocess_image_scores(os.path.join(REF, "datasets", "kodak"), out_file)
        ref_scores = torch.load(out_file, weights_only=True).numpy()
    ours = np.stack([so.image_scores(grays[os.path.abspath(f)]) for f in files])
    np.testing.assert_array_equal(ours, ref_scores)  # exact-integer judge == the reference's float64 judge here
    rgb = np.stack([np.array(Image.open(f).convert("RGB").resize((224, 224), Image.BICUBIC)) for f in files])
    pick = [0, 3, 14, 17]  # two landscape 768x512, two portrait 512x768
    np.savez_compressed(os.path.join(OUT, "kodak.npz"), names=np.array([os.path.basename(f) for f in files]),
                        rgb224=rgb, scores=ref_scores.astype(np.float32), gray_idx=np.array(pick),
                        **{f"gray{i}": grays[os.path.abspath(files[i])] for i in pick})
    print("kodak: scores", ref_scores.shape, "rgb", rgb.shape, "gray", [grays[os.path.abspath(files[i])].shape for i in pick])


if __name__ == "__main__":
    huffman_golden()
    kodak_golden()
