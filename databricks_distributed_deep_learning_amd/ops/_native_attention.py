"""Attention binding (interim: SDPA until attention.hip lands)."""
from .attention import attention_reference


def attention(qkv, num_heads, mask, dropout_p):
    return attention_reference(qkv, num_heads, mask, dropout_p, dropout_p > 0)
