"""ResNet-18/34/50/101/152 (v1.5, stride on the 3x3) in NHWC.

Architecturally identical to ``torchvision.models.resnet50`` (the model the
reference loads at ``notebooks/cv/onnx_experiments.py:19``): 25,557,032
parameters, 53 conv + 53 BN for ResNet-50.  Written from scratch (torchvision is
not installed) around the fused ops:

* every conv is followed by a BatchNorm that fuses ReLU, and the last BN of a
  block also fuses the residual add (``bn3(conv3(x), residual=identity)``), so
  one bottleneck is 3 conv + 3 fused BN launches (+1 conv/BN for downsample);
* activations are NHWC end to end; the model accepts NCHW inputs too
  (``channels_last_input=False``) and permutes once at the stem.
"""
from __future__ import annotations

import os
from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from .. import ops
from ..ops.bridge import GradBridge
from .layers import BatchNorm2d, Conv2d, Linear, conv_bn, conv_bn_add_bn, conv_bn_maxpool, conv_stats


_BRIDGE = os.environ.get("DDL_GRAD_BRIDGE", "1") != "0"


def _bridge(x: torch.Tensor, training: bool):
    return GradBridge() if (_BRIDGE and training and torch.is_grad_enabled() and x.requires_grad) else None


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 zero_init_residual: bool = False):
        super().__init__()
        self.conv1 = Conv2d(cin, planes, 3, stride, 1)
        self.bn1 = BatchNorm2d(planes, relu=True)
        self.conv2 = Conv2d(planes, planes, 3, 1, 1)
        self.bn2 = BatchNorm2d(planes, relu=True, zero_init=zero_init_residual)
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is None:
            br = _bridge(x, self.training)
            out = conv_bn(self.conv1, self.bn1, x, grad_residual=br)
            return conv_bn(self.conv2, self.bn2, out, residual=x, residual_grad_to=br)
        br = _bridge(x, self.training)
        y_id, st_id = self.downsample.conv_stats(x, grad_residual=br)
        out = conv_bn(self.conv1, self.bn1, x, grad_to=br)
        return conv_bn_add_bn(self.conv2, self.bn2, out, self.downsample.bn, y_id, st_id)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 zero_init_residual: bool = False):
        super().__init__()
        self.conv1 = Conv2d(cin, planes, 1)
        self.bn1 = BatchNorm2d(planes, relu=True)
        self.conv2 = Conv2d(planes, planes, 3, stride, 1)
        self.bn2 = BatchNorm2d(planes, relu=True)
        self.conv3 = Conv2d(planes, planes * 4, 1)
        self.bn3 = BatchNorm2d(planes * 4, relu=True, zero_init=zero_init_residual)
        self.downsample = downsample

    def forward(self, x):
        # every conv -> BN pair takes its BN statistics from the conv's GEMM epilogue
        if self.downsample is None:
            # identity block: the residual gradient is added inside conv1's dgrad epilogue
            br = _bridge(x, self.training)
            out = conv_bn(self.conv1, self.bn1, x, grad_residual=br)
            out = conv_bn(self.conv2, self.bn2, out)
            return conv_bn(self.conv3, self.bn3, out, residual=x, residual_grad_to=br)
        # downsample block: conv1 offers its input gradient to the downsample conv,
        # whose dgrad epilogue adds it (autograd runs the longer conv1 branch first)
        # (its BatchNorm is applied together with bn3's: conv_bn_add_bn)
        br = _bridge(x, self.training)
        y_id, st_id = self.downsample.conv_stats(x, grad_residual=br)
        out = conv_bn(self.conv1, self.bn1, x, grad_to=br)
        out = conv_bn(self.conv2, self.bn2, out)
        return conv_bn_add_bn(self.conv3, self.bn3, out, self.downsample.bn, y_id, st_id)


class Downsample(nn.Module):
    """1x1 strided conv + BN (torchvision's ``downsample`` Sequential, same keys 0/1)."""

    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.add_module("0", Conv2d(cin, cout, 1, stride, 0))
        self.add_module("1", BatchNorm2d(cout, relu=False))

    @property
    def bn(self):
        return self._modules["1"]

    def conv_stats(self, x, grad_residual=None):
        """The strided conv with its BatchNorm's statistics partials; the BN is applied by the
        block together with the main branch's last BN (``conv_bn_add_bn``)."""
        return conv_stats(self._modules["0"], self._modules["1"], x, grad_residual=grad_residual)

    def forward(self, x, grad_residual=None):
        return conv_bn(self._modules["0"], self._modules["1"], x, grad_residual=grad_residual)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False, channels_last_input: bool = True):
        super().__init__()
        self.channels_last_input = channels_last_input
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, 7, 2, 3)
        self.bn1 = BatchNorm2d(64, relu=True)
        self.layer1 = self._make_layer(block, 64, layers[0], 1, zero_init_residual)
        self.layer2 = self._make_layer(block, 128, layers[1], 2, zero_init_residual)
        self.layer3 = self._make_layer(block, 256, layers[2], 2, zero_init_residual)
        self.layer4 = self._make_layer(block, 512, layers[3], 2, zero_init_residual)
        self.fc = Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride, zir):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = Downsample(self.inplanes, planes * block.expansion, stride)
        mods = [block(self.inplanes, planes, stride, down, zir)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            mods.append(block(self.inplanes, planes, 1, None, zir))
        return nn.Sequential(*mods)

    # ZeRO-1 gather waits (parallel/ddp.py): the root's forward reads the stem's conv / BN
    # directly (conv_bn_maxpool), every other parameter through a child's forward
    _ddl_direct_reads = ("conv1", "bn1")

    def features(self, x):
        if not self.channels_last_input:
            x = x.permute(0, 2, 3, 1).contiguous()
        x = conv_bn_maxpool(self.conv1, self.bn1, x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return ops.global_avg_pool(x)

    def forward(self, x):
        return self.fc(self.features(x))


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, **kw)


def resnet152(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, **kw)


def from_torchvision_state_dict(sd: dict) -> dict:
    """Convert a torchvision ResNet state dict (OIHW convs) to this layout."""
    out = {}
    for k, v in sd.items():
        if v.dim() == 4:
            v = v.permute(0, 2, 3, 1).contiguous()
        out[k] = v
    return out


def to_torchvision_state_dict(sd: dict) -> dict:
    out = {}
    for k, v in sd.items():
        if v.dim() == 4:
            v = v.permute(0, 3, 1, 2).contiguous()
        out[k] = v
    return out
