"""Synthetic DIV2K-shaped training set for the data-parallel training step (BASELINE config 3,
SURVEY §8(d)).

The reference trains from an image folder through ``get_image_dataset`` (utils/dataloader.py:47-78)
and a ``DistributedSampler`` (training.py:122-129), seeding each process with ``args.seed + rank``
(training.py:109-110).  There is no network here, so config 3 stands in DIV2K's shape: per rank, a
few seeded uint8 noise images of 2040 x 1356 (DIV2K's landscape size), kept resident in HBM, and every
sample is a random 256 x 256 crop of one of them, converted like the loader's ToTensor + Normalize
(dataloader.py:58-61) by one device kernel (``ops.crop_normalize_u8``).  Crop positions and patch
scores are drawn up front from a host generator seeded with ``seed + rank``, so the timed steps do
no host work and no host synchronisation.
"""
from __future__ import annotations

import torch

from . import ops

DIV2K_HW = (1356, 2040)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class SyntheticCropSet:
    def __init__(self, device, seed: int, rank: int = 0, num_images: int = 16, crop: int = 256,
                 patch_size: int = 16, hw=DIV2K_HW):
        self.device = torch.device(device)
        self.crop, self.hw = crop, hw
        self.L = (crop // patch_size) ** 2
        self.gen = torch.Generator().manual_seed(seed + rank)
        H, W = hw
        src = torch.randint(0, 256, (num_images, H, W, 3), dtype=torch.uint8, generator=self.gen)
        self.images = src.to(self.device)
        self._plan = None
        self._i = 0

    def plan(self, steps: int, batch: int):
        """draw `steps` batches of (image, top, left) crops and patch scores; uploaded once"""
        H, W = self.hw
        n = self.images.shape[0]
        c = torch.stack([torch.randint(0, n, (steps, batch), generator=self.gen),
                         torch.randint(0, H - self.crop + 1, (steps, batch), generator=self.gen),
                         torch.randint(0, W - self.crop + 1, (steps, batch), generator=self.gen)], dim=-1)
        scores = torch.rand(steps, batch, self.L, generator=self.gen)
        self._plan = (c.to(torch.int32).to(self.device), scores.to(self.device))
        self._i = 0
        self._out = [torch.empty((batch, 3, self.crop, self.crop), dtype=torch.float32, device=self.device)
                     for _ in range(2)]
        return self

    def next(self):
        """the next planned batch: (imgs [B, 3, crop, crop] f32 normalised, total_scores [B, L] f32)"""
        crops, scores = self._plan
        n = self._i
        self._i += 1
        i = n % crops.shape[0]
        # two buffers, alternating on the monotonic call count (not the wrapped plan index, which repeats a
        # buffer when an odd-length plan wraps): a batch stays valid while the next one is cut
        out = self._out[n & 1]
        ops.crop_normalize_u8(self.images, crops[i], self.crop, IMAGENET_MEAN, IMAGENET_STD, out=out)
        return out, scores[i]
