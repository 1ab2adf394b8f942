"""ViT-B/16 image classifier (pre-LN), sharing the NLP kernels (BASELINE.json:10).

Equivalent to HF ``ViTForImageClassification`` (86,567,656 params at 1000
classes) with fused QKV; the 16x16/16 patch embedding is a GEMM over
NHWC patches ``[B·196, 16·16·3] x [768, 768]^T`` (weight stored (kh, kw, c)).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from ..ops.bridge import GradBridge
from .layers import Dropout, LayerNorm, Linear

# residual-stream gradient handed to the LayerNorm backwards (False: autograd sums it; tests)
_LN_BRIDGE = True


@dataclass
class ViTConfig:
    image_size: int = 224
    patch_size: int = 16
    num_channels: int = 3
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.0
    attention_probs_dropout_prob: float = 0.0
    initializer_range: float = 0.02
    num_labels: int = 1000


class ViTLayer(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        H, I, std = c.hidden_size, c.intermediate_size, c.initializer_range
        self.num_heads = c.num_attention_heads
        self.attn_dropout = c.attention_probs_dropout_prob
        self.layernorm_before = LayerNorm(H, c.layer_norm_eps)
        self.qkv = Linear(H, 3 * H, init_std=std)
        self.attn_out = Linear(H, H, init_std=std)
        self.layernorm_after = LayerNorm(H, c.layer_norm_eps)
        self.fc1 = Linear(H, I, act="gelu", init_std=std)
        self.fc2 = Linear(I, H, init_std=std)
        self.dropout = Dropout(c.hidden_dropout_prob)
        for lin in (self.qkv, self.attn_out, self.fc1, self.fc2):
            nn.init.zeros_(lin.bias)

    def forward(self, h):
        b1 = GradBridge() if _LN_BRIDGE else None
        y = self.layernorm_before(h, grad_from=b1)
        ctx = ops.attention(self.qkv(y), self.num_heads, None, self.attn_dropout, self.training)
        if self.dropout.p > 0.0 and self.training:
            h = h + self.dropout(self.attn_out(ctx))
            y = self.layernorm_after(h)
            return h + self.dropout(self.fc2(self.fc1(y), fuse_dgelu=True))
        # no hidden dropout (the ViT-B/16 recipe): both residual-stream adds ride the output
        # GEMMs' epilogues; fc2's dgrad epilogue applies fc1's GELU backward.  The residual
        # stream's gradient reaches each LayerNorm backward through a bridge, which adds it
        # to the LN input gradient in the same pass (no autograd add, and the column sums --
        # the producing Linear's bias gradient -- come out of that pass too)
        h = self.attn_out(ctx, residual=h, residual_grad_to=b1)
        b2 = GradBridge() if _LN_BRIDGE else None
        y = self.layernorm_after(h, grad_from=b2)
        return self.fc2(self.fc1(y), fuse_dgelu=True, residual=h, residual_grad_to=b2)


class ViTForImageClassification(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        self.config = c
        P, C, H = c.patch_size, c.num_channels, c.hidden_size
        self.num_patches = (c.image_size // P) ** 2
        self.patch_embed = Linear(P * P * C, H, init_std=c.initializer_range)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, H))
        self.position_embeddings = nn.Parameter(torch.empty(1, self.num_patches + 1, H))
        nn.init.trunc_normal_(self.position_embeddings, std=c.initializer_range)
        nn.init.trunc_normal_(self.cls_token, std=c.initializer_range)
        self.dropout = Dropout(c.hidden_dropout_prob)
        self.layers = nn.ModuleList([ViTLayer(c) for _ in range(c.num_hidden_layers)])
        self.layernorm = LayerNorm(H, c.layer_norm_eps)
        self.classifier = Linear(H, c.num_labels, init_std=c.initializer_range)
        nn.init.zeros_(self.classifier.bias)

    # ZeRO-1 gather waits (parallel/ddp.py): the root's forward reads the patch embedding directly
    _ddl_direct_reads = ("patch_embed",)

    def patchify(self, x):
        """NHWC [B, 224, 224, 3] -> [B, 196, 768] in (kh, kw, c) order."""
        B, Hh, Ww, C = x.shape
        P = self.config.patch_size
        x = x.view(B, Hh // P, P, Ww // P, P, C).permute(0, 1, 3, 2, 4, 5)
        return x.reshape(B, (Hh // P) * (Ww // P), P * P * C)

    def forward(self, x):
        # implicit im2col on the image (ops.patch_embed): no patchify copy on the GPU
        t = ops.patch_embed(x, self.patch_embed.weight, self.patch_embed.bias, self.config.patch_size)
        # [cls | patches] + position embeddings in one native pass (ops/glue.py prepend_token_add)
        t = ops.prepend_token_add(t, self.cls_token.to(t.dtype), self.position_embeddings.to(t.dtype))
        h = self.dropout(t)
        for layer in self.layers:
            h = layer(h)
        h = self.layernorm(h)
        return self.classifier(ops.first_token(h))


def vit_b16(num_classes: int = 1000, dropout: float = 0.0, image_size: int = 224) -> ViTForImageClassification:
    return ViTForImageClassification(ViTConfig(num_labels=num_classes, hidden_dropout_prob=dropout,
                                               attention_probs_dropout_prob=dropout, image_size=image_size))


def from_hf_state_dict(sd: dict, num_layers: int, patch: int = 16) -> dict:
    """HF ``ViTForImageClassification`` -> this model."""
    out = {}
    w = sd["vit.embeddings.patch_embeddings.projection.weight"]      # [768, C, P, P]
    out["patch_embed.weight"] = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
    out["patch_embed.bias"] = sd["vit.embeddings.patch_embeddings.projection.bias"]
    out["cls_token"] = sd["vit.embeddings.cls_token"]
    out["position_embeddings"] = sd["vit.embeddings.position_embeddings"]
    out["layernorm.weight"] = sd["vit.layernorm.weight"]
    out["layernorm.bias"] = sd["vit.layernorm.bias"]
    out["classifier.weight"] = sd["classifier.weight"]
    out["classifier.bias"] = sd["classifier.bias"]
    v5 = any(k.startswith("vit.layers.") for k in sd)   # transformers >= 5 naming
    for i in range(num_layers):
        for t in ("weight", "bias"):
            if v5:
                p = f"vit.layers.{i}."
                qkv = [sd[p + f"attention.{n}_proj.{t}"] for n in ("q", "k", "v")]
                names = {"attn_out": "attention.o_proj", "layernorm_before": "layernorm_before",
                         "layernorm_after": "layernorm_after", "fc1": "mlp.fc1", "fc2": "mlp.fc2"}
            else:
                p = f"vit.encoder.layer.{i}."
                qkv = [sd[p + f"attention.attention.{n}.{t}"] for n in ("query", "key", "value")]
                names = {"attn_out": "attention.output.dense", "layernorm_before": "layernorm_before",
                         "layernorm_after": "layernorm_after", "fc1": "intermediate.dense", "fc2": "output.dense"}
            out[f"layers.{i}.qkv.{t}"] = torch.cat(qkv, 0)
            for ours, theirs in names.items():
                out[f"layers.{i}.{ours}.{t}"] = sd[p + f"{theirs}.{t}"]
    return out
