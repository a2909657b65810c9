"""Patch importance scores — counterpart of reference generate_scores_file.py (preprocess_image_scores,
process_dataset) with utils/map.py and utils/distribution.py: the ``total_scores`` input of
MCM.forward / compress for real images.

The whole producer (quadtree split / merge, Laplacian, both resizes, 16x16 patch means, product and
min-max normalisation) runs on the device (csrc/scores.hip, tmae_image_scores): one launch sequence per
batch of equal-size grayscale images, no host round trip.  The cv2 arithmetic is restated from OpenCV's
algorithms (OpenCV is not in the image; parity with cv2 itself is unpinned); the
quadtree / patch glue is pinned to the reference's own code on the 24 Kodak images
(tools/gen_golden_eval.py, tests/golden/kodak.npz).
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import torch

from . import _lib
from .ops import _stream

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def imread_gray(path) -> np.ndarray:
    """cv2.imread(path, IMREAD_GRAYSCALE), host-side data loading:
      * PNG (and other non-JPEG formats): libpng's rgb_to_gray(0.299, 0.587) 15-bit fixed point, OpenCV's PNG
        decoder path -- pinned against the reference's glue on the 24 Kodak PNGs (tests/golden/kodak.npz);
      * JPEG: OpenCV asks libjpeg for JCS_GRAYSCALE output, i.e. the decoded luma plane without colour
        conversion; PIL's ``draft('L')`` requests the same libjpeg output.  cv2 is absent here, so JPEG
        parity is UNPINNED (no fixture covers it)."""
    from PIL import Image

    im = Image.open(path)
    if im.format == "JPEG" and im.mode in ("RGB", "YCbCr"):
        im.draft("L", im.size)  # libjpeg grayscale output at full scale (no DCT downscaling)
    if im.mode == "L":
        return np.array(im)
    rgb = np.array(im.convert("RGB")).astype(np.int64)
    return ((9798 * rgb[..., 0] + 19235 * rgb[..., 1] + 3735 * rgb[..., 2] + 16384) >> 15).astype(np.uint8)


def image_scores(gray: torch.Tensor, size: int = 224, patch: int = 16) -> torch.Tensor:
    """gray: uint8 device tensor [n, H, W] (or [H, W]) -> f32 scores [n, (size / patch)^2] on the device"""
    g = gray.unsqueeze(0) if gray.dim() == 2 else gray
    if g.dtype != torch.uint8 or not g.is_cuda:
        raise ValueError("image_scores needs a uint8 device tensor [n, H, W]")
    g = g.contiguous()
    n, H, W = g.shape
    work = torch.empty(int(_lib.value("tmae_image_scores_workspace", n, H, W, size)), dtype=torch.uint8,
                       device=g.device)
    out = torch.empty((n, (size // patch) ** 2), dtype=torch.float32, device=g.device)
    _lib.call("tmae_image_scores", g.data_ptr(), n, H, W, size, patch, work.data_ptr(), work.numel(), out.data_ptr(),
              _stream())
    return out


def preprocess_image_scores(images, size: int = 224, device="cuda") -> torch.Tensor:
    """generate_scores_file.py:13-36: score every image (paths or grayscale uint8 arrays), images of one
    shape batched into one device call; returns f32 [N, L] on the CPU in input order (torch.save-able)."""
    grays = [imread_gray(p) if isinstance(p, (str, Path)) else np.asarray(p, dtype=np.uint8) for p in images]
    out = [None] * len(grays)
    by_shape = {}
    for i, g in enumerate(grays):
        by_shape.setdefault(g.shape, []).append(i)
    for shape, idx in by_shape.items():
        batch = torch.from_numpy(np.stack([grays[i] for i in idx])).to(device)
        sc = image_scores(batch, size).cpu()
        for j, i in enumerate(idx):
            out[i] = sc[j]
    return torch.stack(out)


def process_dataset(mode, dataset_path, size: int = 224):
    """generate_scores_file.py:39-52: writes <dataset>_scores/<mode>.pt next to the dataset"""
    dataset_path = Path(dataset_path)
    root = dataset_path if mode == "test" else dataset_path / mode
    files = sorted(p for p in root.rglob("*.*") if p.suffix.lower() in IMG_EXTENSIONS)
    out_dir = dataset_path.parent / f"{dataset_path.name}_scores"
    out_dir.mkdir(parents=True, exist_ok=True)
    scores = preprocess_image_scores(files, size)
    torch.save(scores, os.path.join(out_dir, f"{mode}.pt"))
    return scores
