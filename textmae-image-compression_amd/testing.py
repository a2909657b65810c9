"""Kodak evaluation harness — counterpart of reference testing.py: load a checkpoint,
``update(force=True)``, then per image compress -> Huffman-code ids_restore (side info) -> decompress ->
PSNR / MS-SSIM / bpp / encode and decode times, averaged, printed and written as report.txt JSON.

Same function names and arithmetic as the reference (testing.py:40-165, 199-250):
  * compute_metrics: both images rounded to 0..255, PSNR over the batch (psnr, testing.py:40-41),
    pytorch_msssim ms_ssim with data_range 255 -- both on the device (csrc/metrics.hip);
  * bpp = 8 * sum(len(s[0]) for s in strings) / pixels + len(huffman_bits) / pixels (testing.py:88-89):
    the y string plus ONLY the first image's z string (s[0] of the z list), as the reference counts it;
  * batch 1, the test transform (PIL bicubic resize to 224, ToTensor; no normalisation,
    utils/dataloader.py:69-73), scores from <dataset>_scores/test.pt or, when absent, from the device
    score-map producer (scores.py) instead of the reference's RuntimeError (dataloader.py:30-31).
Deviation: ``inference_entropy_estimation`` takes the scores (the reference calls model.forward(x) without
them, testing.py:106, which raises).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import defaultdict
from pathlib import Path

import numpy as np
import torch

from . import _lib, ops
from .huffman import HuffmanCoding
from .ops import _stream

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def collect_images(rootpath):
    files = []
    for ext in IMG_EXTENSIONS:
        files.extend(Path(rootpath).rglob(f"*{ext}"))
    return sorted(files)


def compute_metrics(org: torch.Tensor, rec: torch.Tensor, max_val: int = 255):
    """testing.py:44-49 -> {"psnr", "ms-ssim"} (device kernels; one D2H read of two floats)"""
    if max_val != 255:
        raise ValueError("compute_metrics: the reference evaluates at max_val=255")
    a = org.detach().float().contiguous()
    b = rec.detach().float().contiguous()
    if a.shape != b.shape or not a.is_cuda:
        raise ValueError("compute_metrics needs two device tensors of one shape")
    n, C, H, W = a.shape
    work = torch.empty(int(_lib.value("tmae_metrics_workspace", n, C, H, W)), dtype=torch.float32, device=a.device)
    out = torch.empty(2, dtype=torch.float32, device=a.device)
    _lib.call("tmae_image_metrics", a.data_ptr(), b.data_ptr(), n, C, H, W, work.data_ptr(), work.numel(),
              out.data_ptr(), _stream())
    v = out.tolist()
    return {"psnr": v[0], "ms-ssim": v[1]}


def bits_per_pixel(strings, huffman_bits, num_pixels):
    """testing.py:88-89 (the s[0] of each string list: the y string and the first z string)"""
    return sum(len(s[0]) for s in strings) * 8.0 / num_pixels + len(huffman_bits) / num_pixels


def save_output(x, ori_shape, file_name, output_dir):
    """testing.py:52-57 (the resized image is discarded there too: the saved file is the 224^2 output)"""
    from PIL import Image

    a = x.squeeze().clamp(0, 1).mul(255).round().byte().permute(1, 2, 0).cpu().numpy()
    Image.fromarray(a).save(os.path.join(output_dir, file_name))


@torch.no_grad()
def inference(model, x, ori_shape, total_score, file_name=None, output_dir=None):
    """testing.py:60-100"""
    device = next(model.parameters()).device
    x = x.to(device)
    total_score = total_score.to(device)
    torch.cuda.synchronize()
    start = time.time()
    out_enc = model.compress(x, total_score)
    enc_time = time.time() - start
    ids_keep = out_enc["ids_restore"]
    huffman = HuffmanCoding()
    compressed_ids_keep, shape, dev = huffman.compress(ids_keep)
    decompressed_ids_keep = huffman.decompress(compressed_ids_keep, shape, dev)
    start = time.time()
    out_dec = model.decompress(out_enc["string"], out_enc["shape"], decompressed_ids_keep)
    torch.cuda.synchronize()
    dec_time = time.time() - start
    metrics = compute_metrics(x, out_dec["x_hat"], 255)
    num_pixels = x.size(0) * x.size(2) * x.size(3)
    bpp = bits_per_pixel(out_enc["string"], compressed_ids_keep, num_pixels)
    if output_dir is not None and file_name is not None:
        save_output(out_dec["x_hat"], ori_shape, file_name, output_dir)
    return {"psnr": metrics["psnr"], "ms-ssim": metrics["ms-ssim"], "bpp": bpp, "encoding_time": enc_time,
            "decoding_time": dec_time}


@torch.no_grad()
def inference_entropy_estimation(model, x, total_score):
    """testing.py:103-120 with the scores passed (the reference omits them and raises)"""
    device = next(model.parameters()).device
    x, total_score = x.to(device), total_score.to(device)
    torch.cuda.synchronize()
    start = time.time()
    out = model.forward(x, total_score)
    torch.cuda.synchronize()
    elapsed = time.time() - start
    metrics = compute_metrics(x, out["x_hat"], 255)
    num_pixels = x.size(0) * x.size(2) * x.size(3)
    bpp = float(ops.bpp(out["likelihoods"]["y"], out["likelihoods"]["z"], num_pixels))  # device reduction
    return {"psnr": metrics["psnr"], "ms-ssim": metrics["ms-ssim"], "bpp": bpp, "encoding_time": elapsed / 2.0,
            "decoding_time": elapsed / 2.0}


def load_test_images(paths, size=224):
    """the test transform (utils/dataloader.py:69-73): RGB, PIL bicubic resize to size^2, ToTensor"""
    from PIL import Image

    out = []
    for p in paths:
        im = Image.open(p).convert("RGB")
        ori = im.size
        a = np.array(im.resize((size, size), Image.BICUBIC), dtype=np.float32) / 255.0
        out.append((torch.from_numpy(a).permute(2, 0, 1).unsqueeze(0).contiguous(), ori))
    return out


def eval_model(model, output_dir, images, scores, names=None, entropy_estimation=False):
    """testing.py:128-165 over pre-loaded (img [1,3,S,S], orig_shape) pairs and a [N, L] score tensor"""
    metrics = defaultdict(float)
    if output_dir is not None:
        os.makedirs(output_dir, exist_ok=True)
    for i, (img, ori_shape) in enumerate(images):
        ts = scores[i:i + 1]
        if entropy_estimation:
            rv = inference_entropy_estimation(model, img, ts)
        else:
            rv = inference(model, img, ori_shape, ts, None if names is None else names[i], output_dir)
        for k, v in rv.items():
            metrics[k] += v
    for k in metrics:
        metrics[k] /= len(images)
    return dict(metrics)


def load_checkpoint(num_keep_patches, checkpoint_path, img_size=224, **model_kwargs):
    """testing.py:123-125: the checkpoint's 'model' state_dict into MCM.from_state_dict (CDF buffers resized
    by the compressai-style load_state_dict).  Loaded with weights_only=True; the reference's save_model
    (models/Compression/common/model_utils.py:30-55) stores ``args`` as an argparse.Namespace next to the
    model, so that one class is allow-listed for the weights-only unpickler."""
    from .mcm import MCM

    with torch.serialization.safe_globals([argparse.Namespace]):
        sd = torch.load(checkpoint_path, map_location="cpu", weights_only=True)["model"]
    net = MCM(img_size=img_size, num_keep_patches=num_keep_patches, **model_kwargs)
    net.load_state_dict(sd)
    return net.eval()


def setup_args():
    p = argparse.ArgumentParser()
    p.add_argument("-d", "--dataset", type=str, help="Path to the dataset")
    p.add_argument("-o", "--output_path", type=str, default="reconstruction")
    p.add_argument("-e", "--entropy-coder", default="ans", choices=["ans"])
    p.add_argument("--cuda", action="store_true")
    p.add_argument("--half", action="store_true", help="bf16 operands (the MI355X counterpart of --half)")
    p.add_argument("--entropy-estimation", action="store_true")
    p.add_argument("-v", "--verbose", action="store_true")
    p.add_argument("-c", "--checkpoint", dest="checkpoint_paths", type=str, nargs="*", required=True)
    p.add_argument("--num_keep_patches", type=int, default=144, required=True)
    p.add_argument("--input_size", type=int, default=224, required=True)
    return p


def main(argv):
    args = setup_args().parse_args(argv)
    filepaths = collect_images(args.dataset)
    if not filepaths:
        print("Error: no images found in directory.", file=sys.stderr)
        sys.exit(1)
    ds = Path(args.dataset)
    score_file = ds.parent / f"{ds.name}_scores" / "test.pt"
    if score_file.exists():
        scores = torch.load(score_file, map_location="cpu", weights_only=True)
    else:
        from .scores import preprocess_image_scores

        scores = preprocess_image_scores(filepaths, args.input_size)
    images = load_test_images(filepaths, args.input_size)
    results = defaultdict(list)
    for run in args.checkpoint_paths:
        model = load_checkpoint(args.num_keep_patches, run, args.input_size).to("cuda")
        if args.half:
            model.compute_dtype = torch.bfloat16
        model.update(force=True)
        m = eval_model(model, args.output_path, images, scores, [p.name for p in filepaths], args.entropy_estimation)
        for k, v in m.items():
            results[k].append(v)
    desc = "entropy estimation" if args.entropy_estimation else args.entropy_coder
    output = {"name": "MCM", "description": f"Inference ({desc})", "results": results}
    print(json.dumps(output, indent=2))
    os.makedirs(args.output_path, exist_ok=True)
    with open(os.path.join(args.output_path, "report.txt"), "w") as f:
        json.dump(output, f, indent=2)
    return output


if __name__ == "__main__":
    main(sys.argv[1:])
