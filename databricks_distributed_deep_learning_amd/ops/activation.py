"""Elementwise activations and dropout (kernel families K17/K18)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def gelu(x: torch.Tensor) -> torch.Tensor:
    """erf-form GELU (BERT's ``hidden_act='gelu'``)."""
    if _lib.use_native(x):
        from . import _native_elementwise
        return _native_elementwise.gelu(x)
    return F.gelu(x)


def relu(x: torch.Tensor) -> torch.Tensor:
    return torch.relu(x)


def dropout(x: torch.Tensor, p: float, training: bool = True) -> torch.Tensor:
    """Inverted dropout.  The HIP path draws its mask from a counter-based hash
    (seed, element index) and regenerates it in backward instead of storing it."""
    if not training or p <= 0.0:
        return x
    if _lib.use_native(x):
        from . import _native_elementwise
        return _native_elementwise.dropout(x, p)
    return F.dropout(x, p, True)
