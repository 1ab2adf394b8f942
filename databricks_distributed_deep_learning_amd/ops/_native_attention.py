"""Fused multi-head attention on MFMA (csrc/kernels/attention.hip), with autograd.

Reads the packed QKV projection in place and writes the packed dQKV gradient, so
no head split / merge copies exist on either pass.  Head dim 64 (BERT-base/large,
ViT-B/16); other head dims use the reference path.
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib
from ._lib import F as CF, I, L, P, U64
from ._native_elementwise import new_seed

_lib.register({
    "ddl_attn_fwd": [P, P, P, P, I, I, I, CF, CF, U64, P, P],
    "ddl_attn_bwd": [P, P, P, P, P, P, P, I, I, I, CF, CF, P, P, P],
    "ddl_attn_dmask_words": [I, I, I],
})

# the fused backward (S <= 128) also writes per-batch column sums of dQKV, from which the QKV
# Linear takes its bias gradient instead of another pass over dQKV (DDL_ATTN_COLSUM=0: off)
_COLSUM = os.environ.get("DDL_ATTN_COLSUM", "1") != "0"
# measurement only (never a training setting): DDL_ATTN_NODROP_DEBUG=1 drops the attention-
# probability dropout, to price its in-kernel mask generation in an A/B run
_NODROP_DEBUG = os.environ.get("DDL_ATTN_NODROP_DEBUG", "0") == "1"


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, num_heads, mask, p_drop):
        qkv = qkv.contiguous()
        B, S, three_hd = qkv.shape
        H = num_heads
        D = three_hd // (3 * H)
        scale = 1.0 / math.sqrt(D)
        out = torch.empty(B, S, H * D, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B, H, S, dtype=torch.float32, device=qkv.device)
        m = None if mask is None else mask.to(torch.float32).reshape(B, S).contiguous()
        seed = new_seed() if p_drop > 0 else 0
        # dropout: the forward draws the keep decisions and stores them as bits (1 per score);
        # the backward reads them instead of regenerating them
        dmask = None
        if p_drop > 0:
            fn = _lib.fn("ddl_attn_dmask_words")
            fn.restype = L
            dmask = torch.empty(fn(B, S, H), dtype=torch.int32, device=qkv.device)
        _lib.call("ddl_attn_fwd", qkv.data_ptr(), _lib.p(m), out.data_ptr(), lse.data_ptr(), B, S, H, scale,
                  float(p_drop), seed, _lib.p(dmask))
        ctx.meta = (B, S, H, scale, float(p_drop), seed)
        ctx.save_for_backward(qkv, out, lse, m, dmask)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, m, dmask = ctx.saved_tensors
        B, S, H, scale, p_drop, seed = ctx.meta
        dout = dout.contiguous()
        delta = torch.empty(B, H, S, dtype=torch.float32, device=qkv.device)
        dqkv = torch.empty_like(qkv)
        # QKV bias gradient rows: per batch (single-workgroup kernels) or per batch and 16-row group
        # (tiled backward kernels: 64-row workgroups of 4 waves)
        tiled_rows = B * 4 * -(-S // 64)
        cs = torch.empty(tiled_rows, 3 * H * 64, dtype=torch.float32, device=qkv.device) if _COLSUM else None
        rc = _lib.fn("ddl_attn_bwd")(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), _lib.p(m),
                                     delta.data_ptr(), dqkv.data_ptr(), B, S, H, scale, p_drop, _lib.p(dmask),
                                     _lib.p(cs), _lib.stream())
        if rc not in (0, 2):
            raise RuntimeError(f"native kernel ddl_attn_bwd failed with HIP error {rc}")
        if cs is not None:
            # rides on the gradient: the producing Linear's bias gradient = column sums of these rows
            # (the version guards against autograd accumulating another gradient into dqkv)
            dqkv._ddl_colsum_rows = (cs[:tiled_rows] if rc == 2 else cs[:B], dqkv._version)
        return dqkv, None, None, None


def attention(qkv, num_heads, mask, dropout_p):
    B, S, three_hd = qkv.shape
    if qkv.dtype != torch.bfloat16 or three_hd != 3 * 64 * num_heads:
        from .attention import attention_reference
        return attention_reference(qkv, num_heads, mask, dropout_p, dropout_p > 0)
    return _Attention.apply(qkv, num_heads, mask, 0.0 if _NODROP_DEBUG else float(dropout_p))
