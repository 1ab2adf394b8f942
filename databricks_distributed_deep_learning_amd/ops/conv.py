"""2-D convolution on NHWC activations with [Cout, KH, KW, Cin] weights.

Kernel family K1/K2/K3.  The reference's ResNet-50 forward
(``notebooks/cv/onnx_experiments.py:32,174``) runs these inside ATen/MIOpen; here
the GPU path is an implicit-GEMM MFMA kernel (csrc/kernels/conv_igemm.hip):
M = N·P·Q output pixels, N_gemm = Cout, K = KH·KW·Cin gathered on the fly.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def conv2d_reference(x: torch.Tensor, w: torch.Tensor, stride: int = 1, padding: int = 0) -> torch.Tensor:
    """Plain PyTorch NHWC convolution (CPU oracle / native=off path)."""
    xn = x.permute(0, 3, 1, 2)
    wn = w.permute(0, 3, 1, 2)
    if x.is_cuda:
        xn = xn.contiguous(memory_format=torch.channels_last)
        wn = wn.contiguous(memory_format=torch.channels_last)
    y = F.conv2d(xn, wn, stride=stride, padding=padding)
    return y.permute(0, 2, 3, 1).contiguous()


def conv2d(x: torch.Tensor, w: torch.Tensor, stride: int = 1, padding: int = 0,
           grad_residual=None, bn_stats=None, grad_to=None) -> torch.Tensor:
    """``grad_residual``: a :class:`ops.bridge.GradBridge` whose pending gradient is
    added to this conv's input gradient (fused into the dgrad GEMM epilogue).
    ``grad_to``: a bridge this conv *offers* its input gradient to (a sibling conv of
    the same input adds it in its own dgrad epilogue; native path only).
    ``bn_stats``: a :class:`ops.bridge.BNStats` that receives BatchNorm statistics
    partials of the output from the GEMM epilogue (for the BN that follows)."""
    if _lib.use_native(x):
        from . import _native_conv
        return _native_conv.conv2d(x, w, stride, padding, grad_residual, bn_stats, grad_to)
    from .bridge import join
    return conv2d_reference(join(x, grad_residual), w, stride, padding)


def out_hw(h: int, w: int, k: int, stride: int, padding: int):
    return (h + 2 * padding - k) // stride + 1, (w + 2 * padding - k) // stride + 1


def conv2d_bias_act_reference(x, w, b, stride=1, padding=0, relu=False, residual=None):
    y = conv2d_reference(x.float(), w.float(), stride, padding)
    if b is not None:
        y = y + b.float()
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def conv2d_bias_act(x, w, b, stride=1, padding=0, relu=False, residual=None):
    """Inference-only fused conv (+bias from folded BN) (+residual) (+ReLU)."""
    if _lib.use_native(x) and x.dtype == torch.bfloat16 and w.shape[0] % 8 == 0:
        from . import _native_conv
        return _native_conv.conv2d_bias_act(x, w, b, stride, padding, relu, residual)
    return conv2d_bias_act_reference(x, w, b, stride, padding, relu, residual)


def patch_embed(x: torch.Tensor, w: torch.Tensor, b, patch: int) -> torch.Tensor:
    """ViT patch embedding of an NHWC image with a ``[D, P*P*C]`` weight in (kh, kw, c)
    order: ``[B, H, W, C] -> [B, (H/P)(W/P), D]``.  GPU: implicit-im2col GEMM on the image
    (``_native_conv._PatchEmbed``); otherwise patchify + Linear."""
    if _lib.use_native(x):
        from . import _native_conv
        y = _native_conv.patch_embed(x, w, b, patch)
        if y is not None:
            return y
    from .linear import linear
    B, Hh, Ww, C = x.shape
    t = x.view(B, Hh // patch, patch, Ww // patch, patch, C).permute(0, 1, 3, 2, 4, 5)
    return linear(t.reshape(B, (Hh // patch) * (Ww // patch), patch * patch * C), w, b)
