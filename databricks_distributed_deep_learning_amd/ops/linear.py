"""Dense layer with fused bias + activation epilogue (kernel families K9/K13/K17).

``y = act(x @ W^T + b)`` with W in [out, in] (PyTorch / HF layout).  On MI355X
the GEMM runs on MFMA (csrc/kernels/gemm.hip) with bias and GELU/ReLU/tanh
applied in the epilogue from the fp32 accumulator — no extra pass over the
[tokens, 3072] FFN activation.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib

ACTS = (None, "gelu", "relu", "tanh")


def _act(y: torch.Tensor, act: Optional[str]) -> torch.Tensor:
    if act is None:
        return y
    if act == "gelu":
        return F.gelu(y)
    if act == "relu":
        return torch.relu(y)
    if act == "tanh":
        return torch.tanh(y)
    raise ValueError(act)


def linear_reference(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
                     act: Optional[str] = None) -> torch.Tensor:
    if x.is_cuda or x.dtype == torch.float32:
        y = F.linear(x, w, b)
        return _act(y, act)
    y = F.linear(x.float(), w.float(), b.float() if b is not None else None)
    return _act(y, act).to(x.dtype)


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
           act: Optional[str] = None, grad_residual=None, fuse_dgelu: bool = False,
           residual: Optional[torch.Tensor] = None, residual_grad_to=None) -> torch.Tensor:
    """``grad_residual``: a :class:`ops.bridge.GradBridge` whose pending gradient (a
    post-LN residual branch's) is added to this layer's input gradient inside the
    dgrad GEMM epilogue instead of by an autograd add kernel.
    ``fuse_dgelu``: ``x`` is the output of a ``act="gelu"`` Linear and this layer is its
    only consumer (an FFN) -- this layer's dgrad epilogue then applies that layer's
    dGELU and sums its bias gradient, so the GELU backward pass disappears.
    ``residual``: ``x W^T + b + residual`` (no activation) -- the pre-LN residual stream
    add done in the GEMM epilogue instead of a separate elementwise pass.
    ``residual_grad_to``: a GradBridge that receives the residual's gradient (this
    output's gradient) for the LayerNorm that also consumes ``residual``
    (``layer_norm(grad_from=...)``), instead of autograd summing the two."""
    if act not in ACTS:
        raise ValueError(f"act must be one of {ACTS}")
    if residual is not None and act is not None:
        raise ValueError("linear(residual=...) is the identity-activation epilogue add")
    if _lib.use_native(x):
        from . import _native_linear
        return _native_linear.linear(x, w, b, act, grad_residual, fuse_dgelu, residual, residual_grad_to)
    from .bridge import join
    y = linear_reference(join(x, grad_residual), w, b, act)
    return y if residual is None else y + residual
