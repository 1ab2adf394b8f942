"""Embedding gather / scatter-add bindings (csrc/kernels/elementwise.hip)."""
from __future__ import annotations

import torch

from ._lib import call, dcode, grad_ready, grad_sink, p


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight):
        ids = ids.contiguous().to(torch.int64)
        V, D = weight.shape
        y = torch.empty(*ids.shape, D, dtype=weight.dtype, device=weight.device)
        call("ddl_embedding_fwd", dcode(weight), p(ids), p(weight), p(y), ids.numel(), D)
        ctx.save_for_backward(ids)
        ctx.w_param = weight
        ctx.wshape = (V, D)
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        V, D = ctx.wshape
        dy = dy.contiguous()
        acc = torch.zeros(V, D, dtype=torch.float32, device=dy.device)
        sink = grad_sink(ctx.w_param)
        dw = sink if sink is not None else torch.empty(V, D, dtype=ctx.wdtype, device=dy.device)
        call("ddl_embedding_bwd", dcode(dy), p(ids), p(dy), p(acc), p(dw), ids.numel(), V, D, int(sink is not None))
        if sink is not None:
            grad_ready(ctx.w_param)
            return None, None
        return None, dw


def embedding(ids, weight):
    if weight.shape[1] % 8 or weight.dtype not in (torch.bfloat16, torch.float32):
        import torch.nn.functional as F
        return F.embedding(ids, weight)
    return _Embedding.apply(ids, weight)
