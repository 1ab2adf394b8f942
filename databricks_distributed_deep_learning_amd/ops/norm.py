"""BatchNorm (+ReLU, +residual add) over NHWC and LayerNorm (+residual add).

Kernel families K4/K5/K6 (BN statistics, fused apply+act, fused backward) and
K16 (LayerNorm fwd/bwd) — SURVEY §2.3.  BatchNorm normalises over every axis but
the last (channels innermost), LayerNorm over the last axis only.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib


# ----------------------------------------------------------------- BatchNorm
def batch_norm_reference(x, weight, bias, running_mean, running_var, training: bool,
                         momentum: float = 0.1, eps: float = 1e-5, relu: bool = False,
                         residual: Optional[torch.Tensor] = None):
    C = x.shape[-1]
    xf = x.reshape(-1, C)
    if training:
        y = F.batch_norm(xf.float(), running_mean, running_var, weight.float() if weight is not None else None,
                         bias.float() if bias is not None else None, True, momentum, eps)
    else:
        y = F.batch_norm(xf.float(), running_mean, running_var, weight.float() if weight is not None else None,
                         bias.float() if bias is not None else None, False, momentum, eps)
    y = y.view_as(x)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def sync_batch_norm_reference(x, weight, bias, running_mean, running_var, momentum: float = 0.1,
                              eps: float = 1e-5, relu: bool = False, residual: Optional[torch.Tensor] = None,
                              group=None):
    """Training-mode BatchNorm whose statistics are summed over ``group`` (SyncBatchNorm).

    Per-channel [sum, sumsq] of every rank are all-reduced (differentiably: the
    backward sums the statistics' gradients over the group too); ranks hold equal
    batch sizes, as in data-parallel training."""
    import torch.distributed as dist
    from torch.distributed.nn.functional import all_reduce
    C = x.shape[-1]
    xf = x.reshape(-1, C).float()
    world = dist.get_world_size(group)
    n = xf.shape[0] * world
    st = all_reduce(torch.cat([xf.sum(0), (xf * xf).sum(0)]), op=dist.ReduceOp.SUM, group=group)
    mean = st[:C] / n
    var = (st[C:] / n - mean * mean).clamp_min(0)
    y = (xf - mean) * torch.rsqrt(var + eps)
    if weight is not None:
        y = y * weight.float() + bias.float()
    with torch.no_grad():
        running_mean.mul_(1 - momentum).add_(mean.detach(), alpha=momentum)
        running_var.mul_(1 - momentum).add_(var.detach() * (n / max(1, n - 1)), alpha=momentum)
    y = y.view_as(x)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def batch_norm(x, weight, bias, running_mean, running_var, training: bool, momentum: float = 0.1,
               eps: float = 1e-5, relu: bool = False, residual: Optional[torch.Tensor] = None,
               residual_grad_to=None, stats=None, group=None):
    """``residual_grad_to``: a :class:`ops.bridge.GradBridge` that receives the
    residual's gradient instead of autograd (see ``ops/bridge.py``).  ``stats``: the
    :class:`ops.bridge.BNStats` the producing conv filled (skips the statistics pass).
    ``group``: a process group -> SyncBatchNorm (statistics summed over its ranks in
    training; one [2C] all-reduce in forward and one in backward per layer)."""
    if _lib.use_native(x):
        from . import _native_norm
        return _native_norm.batch_norm(x, weight, bias, running_mean, running_var, training,
                                       momentum, eps, relu, residual, residual_grad_to, stats, group)
    if training and group is not None:
        return sync_batch_norm_reference(x, weight, bias, running_mean, running_var, momentum, eps, relu,
                                         residual, group)
    return batch_norm_reference(x, weight, bias, running_mean, running_var, training, momentum, eps,
                                relu, residual)


# ----------------------------------------------------------------- LayerNorm
def layer_norm_reference(x, weight, bias, eps: float = 1e-12, residual: Optional[torch.Tensor] = None):
    h = x if residual is None else x + residual
    y = F.layer_norm(h.float(), (h.shape[-1],), weight.float() if weight is not None else None,
                     bias.float() if bias is not None else None, eps)
    return y.to(x.dtype)


def layer_norm(x, weight, bias, eps: float = 1e-12, residual: Optional[torch.Tensor] = None,
               dropout: float = 0.0, residual_grad_to=None, grad_from=None):
    """``LayerNorm(dropout(x) + residual)`` over the last axis; fp32 statistics.

    ``dropout`` (training-time probability on ``x``; post-LN transformers apply it to
    the sublayer output right before the residual add) is fused into the kernels on
    the HIP path: the mask is a counter hash regenerated in the backward, which also
    emits the masked gradient's column sums for the producing Linear's bias.
    ``residual_grad_to``: a :class:`ops.bridge.GradBridge` that receives the residual's
    gradient (for the Linear that also consumes ``residual``) instead of autograd.
    ``grad_from``: a GradBridge holding the gradient of ``x`` from its other consumer (a
    pre-LN block's residual branch, ``linear(residual=x, residual_grad_to=...)``); the
    backward adds it to this LayerNorm's input gradient in the same pass."""
    if _lib.use_native(x):
        from . import _native_norm
        return _native_norm.layer_norm(x, weight, bias, eps, residual, dropout, residual_grad_to, grad_from)
    if dropout > 0.0:
        x = F.dropout(x, dropout, True)
    from .bridge import join
    return layer_norm_reference(join(x, grad_from), weight, bias, eps, residual)


def batch_norm_add_bn(x, weight, bias, running_mean, running_var, momentum, eps, x2, weight2, bias2,
                      running_mean2, running_var2, momentum2, eps2, stats=None, stats2=None):
    """Training ``relu(BN(x) + BN2(x2))`` with both BatchNorms applied in one pass (a ResNet
    downsample block's output).  Returns None when the native kernels do not cover it (CPU, odd
    channel counts): the caller then runs the two BatchNorms separately."""
    if not _lib.use_native(x, x2):
        return None
    from . import _native_norm
    return _native_norm.batch_norm_add_bn(x, weight, bias, running_mean, running_var, momentum, eps, x2, weight2,
                                          bias2, running_mean2, running_var2, momentum2, eps2, stats, stats2)


def bn_relu_maxpool(x, weight, bias, running_mean, running_var, momentum, eps, stats=None):
    """Training ``max_pool2d(relu(BN(x)), 3, 2, 1)`` in one pass over ``x`` (the ResNet stem).
    Returns None when the native kernels do not cover it: the caller runs the ops separately."""
    if not _lib.use_native(x):
        return None
    from . import _native_norm
    return _native_norm.bn_relu_maxpool(x, weight, bias, running_mean, running_var, momentum, eps, stats)
