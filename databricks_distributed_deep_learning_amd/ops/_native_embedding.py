"""Embedding gather / scatter-add bindings (csrc/kernels/elementwise.hip).

The backward sorts the ids (stable) and sums each id's rows in token order with no atomics
(``ddl_embedding_bwd_sorted``): the same gradient bits on every run, and no V x D fp32 buffer
to zero and cast.  ``DDL_EMBED_SORTED=0`` restores the fp32-atomic scatter (A/B timing).
"""
from __future__ import annotations

import os

import torch

from . import _lib
from ._lib import call, dcode, grad_ready, grad_sink, p


_SORTED = os.environ.get("DDL_EMBED_SORTED", "1") != "0"


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
        sink = grad_sink(ctx.w_param)
        n = ids.numel()
        if _SORTED and n > 0:
            # untouched rows: the sink keeps its value (accumulate), a fresh gradient starts at zero
            dw = sink if sink is not None else torch.zeros(V, D, dtype=ctx.wdtype, device=dy.device)
            if _lib.fn("ddl_sort_ids_ok")(n, V):
                # one native launch: a bitonic sort of (id, position) keys in one workgroup's LDS
                s = torch.empty(n, dtype=torch.int32, device=dy.device)
                pi = torch.empty(n, dtype=torch.int64, device=dy.device)
                call("ddl_sort_ids", p(ids), n, p(s), p(pi))
            else:
                # int32 keys (V < 2^31): the radix sort makes half the passes of an int64 one
                s, pi = torch.sort(ids.view(-1).to(torch.int32), stable=True)
            part = torch.empty(2 * ((n + 15) // 16) * D, dtype=torch.float32, device=dy.device)
            call("ddl_embedding_bwd_sorted", dcode(dy), p(s), p(pi), p(dy), p(dw), p(part), n, D,
                 int(sink is not None))
        else:
            acc = torch.zeros(V, D, dtype=torch.float32, device=dy.device)
            dw = sink if sink is not None else torch.empty(V, D, dtype=ctx.wdtype, device=dy.device)
            call("ddl_embedding_bwd", dcode(dy), p(ids), p(dy), p(acc), p(dw), n, V, D, int(sink is not None))
        if sink is not None:
            grad_ready(ctx.w_param)
            return None, None
        return None, dw


def embedding(ids, weight):
    if weight.shape[1] % 8 or weight.dtype not in (torch.bfloat16, torch.float32):
        import torch.nn.functional as F
        return F.embedding(ids, weight)
    return _Embedding.apply(ids, weight)
