"""Fused multi-head attention on MFMA (csrc/kernels/attention.hip), with autograd.

Reads the packed QKV projection in place and writes the packed dQKV gradient, so
no head split / merge copies exist on either pass.  Head dim 64 (BERT-base/large,
ViT-B/16); other head dims use the reference path.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._lib import F as CF, I, L, P, U64
from ._native_elementwise import new_seed

_lib.register({
    "ddl_attn_fwd": [P, P, P, P, I, I, I, CF, CF, U64, P],
    "ddl_attn_bwd": [P, P, P, P, P, P, P, I, I, I, CF, CF, U64, P],
})


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
        _lib.call("ddl_attn_fwd", qkv.data_ptr(), _lib.p(m), out.data_ptr(), lse.data_ptr(), B, S, H, scale,
                  float(p_drop), seed)
        ctx.meta = (B, S, H, scale, float(p_drop), seed)
        ctx.save_for_backward(qkv, out, lse, m)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, m = ctx.saved_tensors
        B, S, H, scale, p_drop, seed = ctx.meta
        dout = dout.contiguous()
        delta = torch.empty(B, H, S, dtype=torch.float32, device=qkv.device)
        dqkv = torch.empty_like(qkv)
        _lib.call("ddl_attn_bwd", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), _lib.p(m),
                  delta.data_ptr(), dqkv.data_ptr(), B, S, H, scale, p_drop, seed)
        return dqkv, None, None, None


def attention(qkv, num_heads, mask, dropout_p):
    B, S, three_hd = qkv.shape
    if qkv.dtype != torch.bfloat16 or three_hd != 3 * 64 * num_heads:
        from .attention import attention_reference
        return attention_reference(qkv, num_heads, mask, dropout_p, dropout_p > 0)
    return _Attention.apply(qkv, num_heads, mask, float(dropout_p))
