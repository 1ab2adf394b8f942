"""Multi-head self-attention core (kernel families K14/K15).

Input is the packed QKV projection ``[B, S, 3·H·D]`` exactly as the fused QKV
GEMM writes it (no permute/copy), output is ``[B, S, H·D]`` ready for the
output projection.  ``mask`` is an optional additive key bias ``[B, S]`` (0 for
keep, large negative for padding), the HF extended-attention-mask convention.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib


def attention_reference(qkv: torch.Tensor, num_heads: int, mask: Optional[torch.Tensor] = None,
                        dropout_p: float = 0.0, training: bool = False) -> torch.Tensor:
    B, S, three_hd = qkv.shape
    hd = three_hd // 3
    D = hd // num_heads
    q, k, v = qkv.view(B, S, 3, num_heads, D).permute(2, 0, 3, 1, 4).unbind(0)
    attn_mask = None
    if mask is not None:
        attn_mask = mask.view(B, 1, 1, S).to(q.dtype if q.is_cuda else torch.float32)
    if q.is_cuda:
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask,
                                           dropout_p=dropout_p if training else 0.0)
    else:
        qf, kf, vf = q.float(), k.float(), v.float()
        s = qf @ kf.transpose(-1, -2) / math.sqrt(D)
        if attn_mask is not None:
            s = s + attn_mask.float()
        p = torch.softmax(s, -1)
        if training and dropout_p > 0:
            p = F.dropout(p, dropout_p, True)
        o = (p @ vf).to(q.dtype)
    return o.permute(0, 2, 1, 3).reshape(B, S, hd)


def attention(qkv: torch.Tensor, num_heads: int, mask: Optional[torch.Tensor] = None,
              dropout_p: float = 0.0, training: bool = False) -> torch.Tensor:
    if _lib.use_native(qkv):
        from . import _native_attention
        return _native_attention.attention(qkv, num_heads, mask, dropout_p if training else 0.0)
    return attention_reference(qkv, num_heads, mask, dropout_p, training)
