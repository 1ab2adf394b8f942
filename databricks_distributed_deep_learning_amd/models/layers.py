"""NN modules over the fused op layer (T-L2 in SURVEY §1.2).

Parameters use the PyTorch/HF names so state dicts map one-to-one onto
torchvision/HF checkpoints (conv weights are stored [Cout, KH, KW, Cin] and
converted on load, see ``models.convert``).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from ..ops.bridge import BNStats


class Conv2d(nn.Module):
    """Bias-free NHWC convolution; weight [Cout, KH, KW, Cin]."""

    def __init__(self, cin: int, cout: int, k: int, stride: int = 1, padding: int = 0):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding = cin, cout, k, stride, padding
        self.weight = nn.Parameter(torch.empty(cout, k, k, cin))
        # kaiming_normal_(mode="fan_out", nonlinearity="relu") as torchvision's ResNet
        std = math.sqrt(2.0 / (cout * k * k))
        nn.init.normal_(self.weight, 0.0, std)

    def forward(self, x, grad_residual=None, bn_stats=None, grad_to=None):
        return ops.conv2d(x, self.weight, self.stride, self.padding, grad_residual=grad_residual, bn_stats=bn_stats,
                          grad_to=grad_to)

    def extra_repr(self):
        return f"{self.cin}, {self.cout}, k={self.k}, stride={self.stride}, padding={self.padding}"


class BatchNorm2d(nn.Module):
    """NHWC BatchNorm with optional fused ReLU and fused residual add.

    Running statistics stay fp32 whatever the compute dtype.
    """

    def __init__(self, c: int, eps: float = 1e-5, momentum: float = 0.1, relu: bool = False,
                 zero_init: bool = False):
        super().__init__()
        self.c, self.eps, self.momentum, self.relu = c, eps, momentum, relu
        self.weight = nn.Parameter(torch.zeros(c) if zero_init else torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self._nbt_pending = 0
        self.sync_group = None      # process group: SyncBatchNorm in training (convert_sync_batchnorm)

    def _flush_nbt(self):
        if self._nbt_pending:
            self.num_batches_tracked.add_(self._nbt_pending)
            self._nbt_pending = 0

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self._flush_nbt()
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        self._nbt_pending = 0
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def forward(self, x, residual: Optional[torch.Tensor] = None, residual_grad_to=None, stats=None):
        if self.training:
            # counted on the host (one tiny kernel per BN per step otherwise); folded into
            # the buffer whenever the state dict is read
            self._nbt_pending += 1
        return ops.batch_norm(x, self.weight, self.bias, self.running_mean, self.running_var,
                              self.training, self.momentum, self.eps, self.relu, residual,
                              residual_grad_to=residual_grad_to, stats=stats, group=self.sync_group)

    def _apply(self, fn, recurse=True):
        # keep running stats in fp32 when the module is cast to bf16
        rm, rv = self.running_mean, self.running_var
        super()._apply(fn, recurse)
        if self.running_mean.dtype != torch.float32:
            self.running_mean = self.running_mean.float()
            self.running_var = self.running_var.float()
        return self

    def extra_repr(self):
        return f"{self.c}, eps={self.eps}, relu={self.relu}"


class Linear(nn.Module):
    def __init__(self, fin: int, fout: int, bias: bool = True, act: Optional[str] = None,
                 init_std: Optional[float] = None):
        super().__init__()
        self.fin, self.fout, self.act = fin, fout, act
        self.weight = nn.Parameter(torch.empty(fout, fin))
        self.bias = nn.Parameter(torch.zeros(fout)) if bias else None
        if init_std is not None:
            nn.init.normal_(self.weight, 0.0, init_std)
        else:
            nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
            if self.bias is not None:
                bound = 1.0 / math.sqrt(fin)
                nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, grad_residual=None, fuse_dgelu: bool = False, residual=None, residual_grad_to=None):
        return ops.linear(x, self.weight, self.bias, self.act, grad_residual=grad_residual, fuse_dgelu=fuse_dgelu,
                          residual=residual, residual_grad_to=residual_grad_to)

    def extra_repr(self):
        return f"{self.fin}, {self.fout}, bias={self.bias is not None}, act={self.act}"


def conv_bn(conv: "Conv2d", bn: "BatchNorm2d", x, residual=None, grad_residual=None, residual_grad_to=None,
            grad_to=None):
    """conv -> BatchNorm(+ReLU)(+residual) with the BN statistics produced by the conv's
    GEMM epilogue in training mode (no separate statistics pass over the conv output)."""
    st = BNStats() if bn.training else None
    y = conv(x, grad_residual=grad_residual, bn_stats=st, grad_to=grad_to)
    return bn(y, residual=residual, residual_grad_to=residual_grad_to, stats=st)


def conv_stats(conv: "Conv2d", bn: "BatchNorm2d", x, grad_residual=None):
    """conv(x) with the BatchNorm statistics partials of ``bn`` from its GEMM epilogue, the
    BatchNorm itself deferred (``conv_bn_add_bn``) -> (y, stats)."""
    st = BNStats() if bn.training else None
    return conv(x, grad_residual=grad_residual, bn_stats=st), st


def conv_bn_add_bn(conv: "Conv2d", bn: "BatchNorm2d", x, bn2: "BatchNorm2d", y2, st2=None):
    """relu(BN(conv(x)) + BN2(y2)), y2 / st2 from ``conv_stats``: a ResNet downsample block's
    output.  In training on the native kernels both BatchNorms are applied in one pass (the
    identity branch's BN output is never written); otherwise BN2's output is BN's residual."""
    st = BNStats() if bn.training else None
    y = conv(x, bn_stats=st)
    if bn.training and bn2.training and bn.sync_group is None and bn2.sync_group is None and bn.relu \
            and not bn2.relu:
        out = ops.batch_norm_add_bn(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                                    y2, bn2.weight, bn2.bias, bn2.running_mean, bn2.running_var, bn2.momentum,
                                    bn2.eps, st, st2)
        if out is not None:
            bn._nbt_pending += 1
            bn2._nbt_pending += 1
            return out
    return bn(y, residual=bn2(y2, stats=st2), stats=st)


def conv_bn_maxpool(conv: "Conv2d", bn: "BatchNorm2d", x):
    """max_pool2d(relu(BN(conv(x))), 3, 2, 1): the ResNet stem.  In training on the native
    kernels the BatchNorm, ReLU and max-pool run as one pass over the conv output."""
    if bn.training and bn.sync_group is None and bn.relu:
        st = BNStats()
        y = conv(x, bn_stats=st)
        out = ops.bn_relu_maxpool(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps, st)
        if out is not None:
            bn._nbt_pending += 1
            return out
        return ops.max_pool2d(bn(y, stats=st), 3, 2, 1)
    return ops.max_pool2d(conv_bn(conv, bn, x), 3, 2, 1)


class LayerNorm(nn.Module):
    def __init__(self, d: int, eps: float = 1e-12):
        super().__init__()
        self.d, self.eps = d, eps
        self.weight = nn.Parameter(torch.ones(d))
        self.bias = nn.Parameter(torch.zeros(d))

    def forward(self, x, residual: Optional[torch.Tensor] = None, dropout: float = 0.0, residual_grad_to=None,
                grad_from=None):
        """``LayerNorm(dropout(x) + residual)``; ``dropout`` only applies in training."""
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual, dropout if self.training else 0.0,
                              residual_grad_to=residual_grad_to, grad_from=grad_from)


class Embedding(nn.Module):
    def __init__(self, n: int, d: int, init_std: float = 0.02):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(n, d))
        nn.init.normal_(self.weight, 0.0, init_std)

    def forward(self, ids):
        return ops.embedding(ids, self.weight)


class Dropout(nn.Module):
    def __init__(self, p: float):
        super().__init__()
        self.p = p

    def forward(self, x):
        return ops.dropout(x, self.p, self.training)


def convert_sync_batchnorm(module: nn.Module, group=None) -> nn.Module:
    """Make every :class:`BatchNorm2d` a SyncBatchNorm over ``group`` (default: the world
    group): training statistics summed across ranks -- one [2C] all-reduce per layer in
    forward and one in backward.  The analogue of ``nn.SyncBatchNorm.convert_sync_batchnorm``."""
    import torch.distributed as dist
    g = group if group is not None else dist.group.WORLD
    for m in module.modules():
        if isinstance(m, BatchNorm2d):
            m.sync_group = g
    return module


def cast_params(module: nn.Module, dtype: torch.dtype) -> nn.Module:
    """Cast parameters (not BN running statistics) to ``dtype``."""
    for m in module.modules():
        for name, p in list(m._parameters.items()):
            if p is not None and p.dtype != dtype and p.is_floating_point():
                m._parameters[name] = nn.Parameter(p.data.to(dtype), requires_grad=p.requires_grad)
    return module
