"""Fused softmax cross-entropy (csrc/kernels/elementwise.hip softmax_ce_k).

Forward computes the per-row loss AND d(mean loss)/d(logits) in one pass over
the logits; backward only rescales by the incoming (device-resident) gradient.
"""
from __future__ import annotations

import torch

from ._lib import call, dcode, p


class _SoftmaxCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        logits = logits.contiguous()
        B, C = logits.shape
        labels = labels.contiguous().to(torch.int64)
        row = torch.empty(B, dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        need_grad = logits.requires_grad
        dl = torch.empty_like(logits) if need_grad else None
        call("ddl_softmax_ce", dcode(logits), p(logits), p(labels), B, C, p(row), p(loss), p(dl))
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        g = g.contiguous().float()
        out = torch.empty_like(dl)
        call("ddl_scale_by", dcode(dl), p(dl), p(g), p(out), dl.numel())
        return out, None


def cross_entropy(logits, labels):
    if logits.dim() != 2 or logits.dtype not in (torch.bfloat16, torch.float32):
        import torch.nn.functional as F
        return F.cross_entropy(logits.float(), labels)
    return _SoftmaxCE.apply(logits, labels)
