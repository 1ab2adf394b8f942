"""Autograd bindings for GELU / dropout (csrc/kernels/elementwise.hip)."""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import call, dcode, p


def new_seed() -> int:
    """Host-side 62-bit seed from torch's CPU generator (no device sync)."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class _Gelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        call("ddl_gelu_fwd", dcode(x), p(x), p(y), x.numel())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        call("ddl_gelu_bwd", dcode(x), p(dy), p(x), p(dx), x.numel())
        return dx


def gelu(x):
    if x.numel() % 8 or x.dtype not in (torch.bfloat16, torch.float32):
        import torch.nn.functional as F
        return F.gelu(x)
    return _Gelu.apply(x)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, prob):
        x = x.contiguous()
        seed = new_seed()
        y = torch.empty_like(x)
        call("ddl_dropout", dcode(x), p(x), p(y), x.numel(), seed, float(prob))
        ctx.seed, ctx.prob = seed, prob
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        call("ddl_dropout", dcode(dy), p(dy), p(dx), dy.numel(), ctx.seed, float(ctx.prob))
        return dx, None


def dropout(x, prob):
    if x.numel() % 8 or x.dtype not in (torch.bfloat16, torch.float32):
        import torch.nn.functional as F
        return F.dropout(x, prob, True)
    return _Dropout.apply(x, prob)


def colsum(x2d: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """out[c] (+)= sum_r x[r, c]  (bias gradients)."""
    from . import _lib
    rows, C = x2d.shape
    nblk = _lib.fn("ddl_colsum_nblk")(rows)
    part = torch.empty(nblk * C, dtype=torch.float32, device=x2d.device)
    call("ddl_colsum", dcode(x2d), p(x2d), rows, C, p(part), p(out), dcode(out), int(accumulate))
    return out


# ------------------------------------------------------------------ step glue (native, no ATen launches)
def tanh_bwd(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """dz = dy * (1 - y^2) from tanh's output."""
    dy, y = dy.contiguous(), y.contiguous()
    dz = torch.empty_like(dy)
    call("ddl_tanh_bwd", dcode(dy), p(dy), p(y), p(dz), dy.numel())
    return dz


def copy2d(dst: torch.Tensor, src: Optional[torch.Tensor], ldd: int, drows: int, dcols: int, lds: int = 0,
           srows: int = 0, scols: int = 0) -> torch.Tensor:
    """dst[r, c] = src[r, c] inside src's (srows x scols) window, 0 elsewhere, for r < drows, c < dcols
    (element strides ldd / lds): zero padding, slicing and strided row gathers in one launch."""
    assert src is None or src.dtype == dst.dtype
    call("ddl_copy2d", dcode(dst), p(dst), ldd, drows, dcols, p(src), lds, srows if src is not None else 0,
         scols if src is not None else 0)
    return dst


def add_into(dst: torch.Tensor, src: torch.Tensor) -> None:
    """dst += src in place (same dtype, contiguous)."""
    assert dst.dtype == src.dtype and dst.numel() == src.numel() and dst.is_contiguous() and src.is_contiguous()
    call("ddl_add_into", dcode(dst), p(dst), p(src), dst.numel())


def zero_(t: torch.Tensor) -> torch.Tensor:
    """Native zero fill of a contiguous tensor."""
    assert t.is_contiguous()
    call("ddl_zero", p(t), t.numel() * t.element_size())
    return t
