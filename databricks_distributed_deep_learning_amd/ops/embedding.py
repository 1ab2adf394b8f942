"""Token embedding gather (K19).  Backward is a scatter-add into the table."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if _lib.use_native(weight):
        from . import _native_embedding
        return _native_embedding.embedding(ids, weight)
    return F.embedding(ids, weight)
