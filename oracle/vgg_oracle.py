"""ORACLE — test infrastructure only.

CPU restatement (plain PyTorch, NCHW) of the reference's VGG16 feature loss: cal_features_loss
(models/Compression/loss/vgg.py:86-115) over torchvision vgg16().features[0:16] (vgg.py:14-29) with
de_normalize / normalize_batch (models/Compression/common/image_utils.py:4-23).  torchvision and its
pretrained weights are absent, so the parity tests use a seeded VGG16 state_dict with torchvision's key
names and shapes (parity with the pretrained network itself is unpinned: the arithmetic is what is checked).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

CFG = [(0, 3, 64), (2, 64, 64), "M", (5, 64, 128), (7, 128, 128), "M", (10, 128, 256), (12, 256, 256), (14, 256, 256)]


def make_vgg_state_dict(seed=0):
    """features.{0,2,5,7,10,12,14}.{weight,bias} with He-scaled random weights (VGG16's first three slices)"""
    rng = np.random.default_rng(seed)
    sd = {}
    for item in CFG:
        if item == "M":
            continue
        i, cin, cout = item
        sd[f"features.{i}.weight"] = torch.from_numpy(
            (rng.standard_normal((cout, cin, 3, 3)) * math.sqrt(2.0 / (9 * cin))).astype(np.float32))
        sd[f"features.{i}.bias"] = torch.from_numpy((0.05 * rng.standard_normal(cout)).astype(np.float32))
    return sd


def features(x, sd):
    """(relu2_2, relu3_3) of Vgg16.forward (vgg.py:34-57)"""
    h, r22 = x, None
    for item in CFG:
        if item == "M":
            h = F.max_pool2d(h, 2, 2)
            continue
        i = item[0]
        h = F.relu(F.conv2d(h, sd[f"features.{i}.weight"].to(h.dtype), sd[f"features.{i}.bias"].to(h.dtype), padding=1))
        if i == 7:
            r22 = h
    return r22, h


def normalize(batch):
    """normalize_batch(de_normalize(batch)) (image_utils.py:4-23)"""
    b = (batch + 1.0) / 2.0 * 255.0
    mean = torch.tensor([0.485, 0.456, 0.406], dtype=b.dtype).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], dtype=b.dtype).view(1, 3, 1, 1)
    return (b / 255.0 - mean) / std


def feature_loss(preds, imgs, sd):
    p22, p33 = features(normalize(preds), sd)
    t22, t33 = features(normalize(imgs), sd)
    return F.mse_loss(p22, t22) + F.mse_loss(p33, t33)
