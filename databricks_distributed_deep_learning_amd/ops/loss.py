"""Softmax cross-entropy (K10) and inference softmax + top-k (K11).

``softmax_topk`` reproduces the reference's post-processing: softmax over the
1000 logits then the 5 best classes (``notebooks/cv/onnx_experiments.py:85-100``
for ORT, ``:174-178`` for PyTorch).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy, fp32 math, returns an fp32 scalar."""
    if _lib.use_native(logits):
        from . import _native_loss
        return _native_loss.cross_entropy(logits, labels)
    return F.cross_entropy(logits.float(), labels)


def softmax_topk(logits: torch.Tensor, k: int = 5):
    """Returns (probabilities, top-k values, top-k indices) over the last axis."""
    p = torch.softmax(logits.float(), dim=-1)
    v, i = torch.topk(p, k, dim=-1)
    return p, v, i
