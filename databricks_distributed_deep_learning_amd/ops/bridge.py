"""Residual-gradient bridge: fold the residual branch's gradient into a GEMM epilogue.

In a ResNet identity block the block input ``x`` feeds both ``conv1`` and the
residual add of the last BatchNorm, so autograd would sum two full-size
gradients with an extra elementwise kernel (read 2, write 1).  With a bridge the
last BN's backward *hands* its residual gradient to the bridge instead of
returning it, and ``conv1``'s backward adds it in the dgrad GEMM epilogue
(``residual=``) -- the sum costs one extra read inside a kernel that runs anyway.

Ordering is guaranteed by data dependence: ``conv1``'s backward needs the
gradient of its output, which only exists after the last BN's backward ran.
A consumer that finds the bridge empty adds nothing (the producer then returned
the gradient to autograd as usual), so mixing native and reference ops stays
correct.

Sibling branches (a downsample block: ``conv1`` and the downsample conv both read
the block input) have no data dependence between their backward passes, so the
producer *offers* its gradient: the offer is refused once the consumer has already
run (``take`` closes the bridge), and the producer then returns the gradient to
autograd itself.  Either execution order sums both gradients exactly once.
"""
from __future__ import annotations

from typing import Optional

import torch


class GradBridge:
    __slots__ = ("grad", "closed")

    def __init__(self):
        self.grad: Optional[torch.Tensor] = None
        self.closed = False

    def put(self, g: torch.Tensor) -> None:
        if self.grad is not None:
            raise RuntimeError("GradBridge: gradient already pending (bridge reused within one backward?)")
        self.grad = g

    def offer(self, g: torch.Tensor) -> bool:
        """Hand ``g`` to the consumer unless it already ran (then the caller keeps it)."""
        if self.closed:
            return False
        self.put(g)
        return True

    def take(self) -> Optional[torch.Tensor]:
        g, self.grad = self.grad, None
        self.closed = True
        return g


class _BridgeJoin(torch.autograd.Function):
    """Identity in forward; adds the bridged gradient in backward (reference-op consumers)."""

    @staticmethod
    def forward(ctx, x, bridge):
        ctx.bridge = bridge
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        r = ctx.bridge.take()
        return (g if r is None else g + r.view_as(g)), None


def join(x: torch.Tensor, bridge: Optional[GradBridge]) -> torch.Tensor:
    return x if bridge is None else _BridgeJoin.apply(x, bridge)


class BNStats:
    """Carries BatchNorm statistics partials from a conv GEMM epilogue to the BN that
    consumes the conv output (forward-time side channel, see ``gemm(colstats=...)``).

    The BN uses them only if they describe exactly the tensor it received (same
    storage pointer and size); otherwise it computes its own statistics."""
    __slots__ = ("ptr", "numel", "part", "nblk")

    def __init__(self):
        self.ptr = None
        self.numel = 0
        self.part = None
        self.nblk = 0

    def set(self, y: torch.Tensor, part: torch.Tensor, nblk: int) -> None:
        self.ptr, self.numel, self.part, self.nblk = y.data_ptr(), y.numel(), part, nblk

    def take_for(self, x: torch.Tensor):
        if self.part is None or self.ptr != x.data_ptr() or self.numel != x.numel():
            return None
        part, nblk = self.part, self.nblk
        self.part = None
        return part, nblk


class BNBackward:
    """Carries a BatchNorm's backward reduction from the dgrad GEMM that produces the
    gradient of the BN output (backward-time side channel, ``gemm(act="bnb")``).

    Set on the BN output in training; the conv that consumes that output finds it on its
    input, applies the BN's ReLU mask in its dgrad epilogue and sums [dz | dz * xhat] per
    column.  The BN uses the partials only if its incoming gradient is exactly that dgrad
    output.  The hint keeps a reference to it, which also stops autograd from accumulating
    a second gradient contribution into it in place (the sum is then a new tensor, the
    pointers differ and the BN computes its own reduction, masking is idempotent)."""
    __slots__ = ("x", "mask", "mean", "istd", "dz", "part", "nrows")

    def __init__(self, x: torch.Tensor, mask: Optional[torch.Tensor], mean: torch.Tensor, istd: torch.Tensor):
        self.x, self.mask, self.mean, self.istd = x, mask, mean, istd
        self.dz = None
        self.part = None
        self.nrows = 0

    def set(self, dz: torch.Tensor, part: torch.Tensor, nrows: int) -> None:
        self.dz, self.part, self.nrows = dz, part, nrows

    def take_for(self, g: torch.Tensor):
        dz, part, nrows = self.dz, self.part, self.nrows
        self.dz = self.part = None
        if dz is None or dz.data_ptr() != g.data_ptr() or dz.numel() != g.numel():
            return None
        return part, nrows
