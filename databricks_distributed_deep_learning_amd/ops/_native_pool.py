"""NHWC max-pool / global-avg-pool bindings (csrc/kernels/elementwise.hip)."""
from __future__ import annotations

import torch

from ._lib import call, dcode, p


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        x = x.contiguous()
        N, H, W, C = x.shape
        P = (H + 2 * pad - k) // s + 1
        Q = (W + 2 * pad - k) // s + 1
        y = torch.empty(N, P, Q, C, dtype=x.dtype, device=x.device)
        idx = torch.empty(N, P, Q, C, dtype=torch.uint8, device=x.device)
        call("ddl_maxpool_fwd", dcode(x), p(x), p(y), p(idx), N, H, W, C, P, Q, k, s, pad)
        ctx.save_for_backward(idx)
        ctx.meta = (N, H, W, C, P, Q, k, s, pad, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, H, W, C, P, Q, k, s, pad, dt = ctx.meta
        dy = dy.contiguous()
        dx = torch.empty(N, H, W, C, dtype=dt, device=dy.device)
        call("ddl_maxpool_bwd", dcode(dy), p(dy), p(idx), p(dx), N, H, W, C, P, Q, k, s, pad)
        return dx, None, None, None


def max_pool2d(x, k=3, stride=2, padding=1):
    if x.shape[-1] % 8 or x.dtype not in (torch.bfloat16, torch.float32) or k * k > 255:
        from .pool import max_pool2d_reference
        return max_pool2d_reference(x, k, stride, padding)
    return _MaxPool.apply(x, k, stride, padding)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty(N, C, dtype=x.dtype, device=x.device)
        call("ddl_avgpool_fwd", dcode(x), p(x), p(y), N, H * W, C)
        ctx.meta = (N, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.meta
        dy = dy.contiguous()
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        call("ddl_avgpool_bwd", dcode(dy), p(dy), p(dx), N, H * W, C)
        return dx


def global_avg_pool(x):
    if x.shape[-1] % 8 or x.dtype not in (torch.bfloat16, torch.float32):
        return x.float().mean(dim=(1, 2)).to(x.dtype)
    return _AvgPool.apply(x)
