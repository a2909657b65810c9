"""ORACLE — test infrastructure only.

CPU restatement of the reference's score-map producer (the input of MCM.get_ids_shuffle):
generate_scores_file.py:19-31 (preprocess_image_scores), utils/map.py:6-60 (quadtree
Division_Merge_Segmented, laplacian), utils/distribution.py:5-16 (cal_patch_score).

PARITY UNPINNED: the reference runs on OpenCV (cv2), which is absent from this image, so its three cv2
calls are restated here from OpenCV 4.x's published algorithms (the x86 build the reference would run):
  * cv2.Laplacian(img, CV_16S, ksize=3): filter2D with the aperture [[2,0,2],[0,-8,0],[2,0,2]],
    BORDER_REFLECT_101; cv2.convertScaleAbs: saturate(|x|) to uint8;
  * cv2.resize(src, (W, H)) INTER_LINEAR on uint8: per output column fx = float((dx + 0.5) * sx - 0.5),
    ix = floor(fx), fx -= ix, clamped at the borders (fx = 0); 11-bit coefficients
    round(w * 2048) (short); horizontal pass exact in int; vertical pass as the SSE2/AVX2 kernel
    VResizeLinearVec_32s8u computes it for full vector widths: (((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16),
    then (x + 2) >> 2 saturated (224 = 14 x 16 = 7 x 32 output columns, no scalar tail);
  * cv2.imread(..., IMREAD_GRAYSCALE) of an RGB PNG: libpng png_set_rgb_to_gray(0.299, 0.587) fixed point,
    gray = (9798 R + 19235 G + 3735 B + 16384) >> 15 (used only to make fixtures).
Division_Judge's float64 mean / std(ddof=1) test `(v - mean) < 2 std` is evaluated exactly in integer
arithmetic ((n v - S)^2 (n - 1) < 4 n (n Sxx - S^2) for v >= mean), which equals numpy's float64
evaluation except for a pixel within float64 rounding of the 2-sigma threshold.
"""
from __future__ import annotations

import math

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS


def rgb_to_gray(rgb: np.ndarray) -> np.ndarray:
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((9798 * r + 19235 * g + 3735 * b + 16384) >> 15).astype(np.uint8)


def _judge(area: np.ndarray) -> bool:
    """Division_Judge (map.py:6-23): fraction of pixels with (v - mean) < 2 std(ddof=1) >= 0.95"""
    v = area.astype(np.int64).reshape(-1)
    n = v.size
    if n < 2:
        return False  # std(ddof=1) of one pixel is NaN: no comparison holds
    S = int(v.sum())
    Q = n * int((v * v).sum()) - S * S  # n^2 (n-1) var
    d = n * v - S                        # n (v - mean)
    below = d < 0
    dd = [int(x) for x in d[~below]]
    ok = int(below.sum()) + sum(1 for x in dd if x * x * (n - 1) < 4 * n * Q)
    return 20 * ok >= 19 * n


def _merge(img, h0, w0, h, w):
    """Merge (map.py:27-31): 60 < v < 150 -> 0, else 255, in place"""
    a = img[h0:h0 + h, w0:w0 + w]
    m = (a > 60) & (a < 150)
    a[m] = 0
    a[~m] = 255


def _recursion(img, h0, w0, h, w):
    """Recursion (map.py:35-42), depth first TL, TR, BL, BR"""
    if not _judge(img[h0:h0 + h, w0:w0 + w]) and min(h, w) > 5:
        h2, w2 = int(h / 2), int(w / 2)
        _recursion(img, h0, w0, h2, w2)
        _recursion(img, h0, w0 + w2, h2, w2)
        _recursion(img, h0 + h2, w0, h2, w2)
        _recursion(img, h0 + h2, w0 + w2, h2, w2)
    else:
        _merge(img, h0, w0, h, w)


def segment(img: np.ndarray) -> np.ndarray:
    """the quadtree split-merge of Division_Merge_Segmented (map.py:46-50) applied IN PLACE to a copy"""
    out = np.array(img, dtype=np.uint8, copy=True)
    _recursion(out, 0, 0, out.shape[0], out.shape[1])
    return out


def _linear_coeffs(ssize: int, dsize: int, clamp: bool):
    """source offsets and 11-bit weights; columns (clamp=True) move a border tap onto the edge with weight
    (1, 0) as resizeGeneric's xofs loop does, rows keep their weights and clip the row index instead"""
    scale = 1.0 / (dsize / ssize)  # scale_x = 1 / inv_scale_x, inv_scale_x = dsize / ssize (double)
    ofs = np.empty(dsize, dtype=np.int64)
    alpha = np.empty((dsize, 2), dtype=np.int64)
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = math.floor(float(f))
        f = np.float32(f - np.float32(s))
        if clamp and s < 0:
            f, s = np.float32(0.0), 0
        if clamp and s >= ssize - 1:
            f, s = np.float32(0.0), ssize - 1
        ofs[d] = s
        a0 = np.float32(np.float32(1.0) - f) * np.float32(COEF_SCALE)
        a1 = f * np.float32(COEF_SCALE)
        alpha[d] = (int(np.rint(a0)), int(np.rint(a1)))
    return ofs, alpha


def resize_linear(src: np.ndarray, W: int, H: int) -> np.ndarray:
    """cv2.resize(src, (W, H)) INTER_LINEAR, uint8 single channel (see the module docstring)"""
    sh, sw = src.shape
    xo, xa = _linear_coeffs(sw, W, True)
    yo, ya = _linear_coeffs(sh, H, False)
    s = src.astype(np.int64)
    x1 = np.minimum(xo + 1, sw - 1)
    hrow = s[:, xo] * xa[:, 0] + s[:, x1] * xa[:, 1]  # [sh][W] int (scale 2048)
    S0, S1 = hrow[np.clip(yo, 0, sh - 1)], hrow[np.clip(yo + 1, 0, sh - 1)]
    b0, b1 = ya[:, 0:1], ya[:, 1:2]
    v = (((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def laplacian_abs(img: np.ndarray) -> np.ndarray:
    """cv2.convertScaleAbs(cv2.Laplacian(img, cv2.CV_16S, ksize=3)) (map.py:56-59 before the resize)"""
    p = np.pad(img.astype(np.int64), 1, mode="reflect")  # numpy 'reflect' == BORDER_REFLECT_101
    c = p[1:-1, 1:-1]
    lap = 2 * (p[:-2, :-2] + p[:-2, 2:] + p[2:, :-2] + p[2:, 2:]) - 8 * c
    return np.minimum(np.abs(lap), 255).astype(np.uint8)


def patch_scores(m: np.ndarray, crop=16, step=16) -> np.ndarray:
    """cal_patch_score (distribution.py:5-16): int(mean) of every 16 x 16 patch, row-major"""
    h, w = m.shape
    return np.array([int(m[x:x + crop, y:y + crop].astype(np.int64).sum()) // (crop * crop)
                     for x in range(0, h - crop + 1, step) for y in range(0, w - crop + 1, step)], dtype=np.int64)


def image_scores(gray: np.ndarray, size: int = 224) -> np.ndarray:
    """preprocess_image_scores body (generate_scores_file.py:19-31) for one grayscale image -> float32 [L].
    Note the reference computes the Laplacian on the image AFTER the in-place merges of the segmentation."""
    seg = segment(gray)
    s_map = resize_linear(seg[1:-1, 1:-1], size, size)
    t_map = resize_linear(laplacian_abs(seg), size, size)
    total = patch_scores(t_map) * patch_scores(s_map)
    with np.errstate(invalid="ignore", divide="ignore"):
        total = (total - total.min()) / (total.max() - total.min())
    return total.astype(np.float32)
