"""Model zoo (N11): ResNet-18/34/50/101/152, BERT-base/large (+ a tiny test size), ViT-B/16."""
from __future__ import annotations

import torch.nn as nn

from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152  # noqa: F401
from .bert import BertConfig, BertForSequenceClassification, bert_base, bert_large, bert_tiny  # noqa: F401
from .vit import ViTConfig, ViTForImageClassification, vit_b16  # noqa: F401
from .layers import cast_params, convert_sync_batchnorm  # noqa: F401

_REGISTRY = {
    "resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50,
    "resnet101": resnet101, "resnet152": resnet152,
    "bert_base": bert_base, "bert_large": bert_large, "bert_tiny": bert_tiny,
    "vit_b16": vit_b16,
}


def available_models():
    return sorted(_REGISTRY)


def build_model(name: str, num_classes: int = 1000, dropout: float = 0.1, image_size: int = 224) -> nn.Module:
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name!r}; have {available_models()}")
    if name.startswith("bert"):
        return _REGISTRY[name](num_labels=num_classes, dropout=dropout)
    if name.startswith("vit"):
        return _REGISTRY[name](num_classes=num_classes, dropout=dropout, image_size=image_size)
    return _REGISTRY[name](num_classes=num_classes)


def count_params(m: nn.Module) -> int:
    return sum(p.numel() for p in m.parameters())
