"""Tensor-space ImageNet preprocessing (reference parity).

The reference preprocesses with ``T.Compose([Resize(256), CenterCrop(224),
ToTensor(), Normalize(mean, std)])`` (``notebooks/cv/onnx_experiments.py:59-64``,
duplicated at :162-167).  torchvision is not installed, so these are
re-implemented on tensors (bilinear resize of the shorter side, antialias off).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn.functional as F

from .synthetic import IMAGENET_MEAN, IMAGENET_STD


def to_tensor(img) -> torch.Tensor:
    """HWC uint8 array / PIL image -> CHW float in [0, 1]."""
    if not isinstance(img, torch.Tensor):
        import numpy as np
        img = torch.from_numpy(np.asarray(img).copy())
    if img.dim() == 2:
        img = img.unsqueeze(-1)
    return img.permute(2, 0, 1).float().div(255.0)


def resize(x: torch.Tensor, size: int) -> torch.Tensor:
    """Resize CHW so the shorter side == size (torchvision ``Resize(int)`` semantics)."""
    c, h, w = x.shape
    if h <= w:
        nh, nw = size, int(size * w / h)
    else:
        nh, nw = int(size * h / w), size
    return F.interpolate(x.unsqueeze(0), size=(nh, nw), mode="bilinear", align_corners=False,
                         antialias=True).squeeze(0)


def center_crop(x: torch.Tensor, size: int) -> torch.Tensor:
    _, h, w = x.shape
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return x[:, top:top + size, left:left + size]


def normalize(x: torch.Tensor, mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD):
    m = torch.tensor(mean, dtype=x.dtype).view(-1, 1, 1)
    s = torch.tensor(std, dtype=x.dtype).view(-1, 1, 1)
    return (x - m) / s


def imagenet_preprocess(img, resize_to: int = 256, crop: int = 224) -> torch.Tensor:
    """Reference pipeline -> CHW float tensor."""
    return normalize(center_crop(resize(to_tensor(img), resize_to), crop))
