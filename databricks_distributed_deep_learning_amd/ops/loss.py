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
    """Returns (probabilities, top-k values, top-k indices) over the last axis.

    On the GPU one HIP kernel does both (softmax_topk_k in elementwise.hip: one block
    per row, probabilities staged in LDS, k block-wide argmax rounds)."""
    if _lib.use_native(logits) and logits.dtype in (torch.bfloat16, torch.float32) and \
            logits.shape[-1] <= 4096 and 1 <= k <= logits.shape[-1]:
        from ._lib import call, dcode, p as ptr
        x = logits.contiguous()
        C = x.shape[-1]
        B = x.numel() // C
        probs = torch.empty(B, C, dtype=torch.float32, device=x.device)
        v = torch.empty(B, k, dtype=torch.float32, device=x.device)
        i = torch.empty(B, k, dtype=torch.int64, device=x.device)
        call("ddl_softmax_topk", dcode(x), ptr(x), B, C, k, ptr(probs), ptr(v), ptr(i))
        lead = x.shape[:-1]
        return probs.view(*lead, C), v.view(*lead, k), i.view(*lead, k)
    p = torch.softmax(logits.float(), dim=-1)
    v, i = torch.topk(p, k, dim=-1)
    return p, v, i
