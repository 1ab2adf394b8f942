"""NHWC pooling: 3x3/2 max-pool (K7) and global average pool (K8)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def max_pool2d_reference(x: torch.Tensor, k: int = 3, stride: int = 2, padding: int = 1) -> torch.Tensor:
    y = F.max_pool2d(x.permute(0, 3, 1, 2), k, stride, padding)
    return y.permute(0, 2, 3, 1).contiguous()


def max_pool2d(x: torch.Tensor, k: int = 3, stride: int = 2, padding: int = 1) -> torch.Tensor:
    if _lib.use_native(x):
        from . import _native_pool
        return _native_pool.max_pool2d(x, k, stride, padding)
    return max_pool2d_reference(x, k, stride, padding)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """[N, H, W, C] -> [N, C] mean over H, W."""
    if _lib.use_native(x):
        from . import _native_pool
        return _native_pool.global_avg_pool(x)
    return x.float().mean(dim=(1, 2)).to(x.dtype)
