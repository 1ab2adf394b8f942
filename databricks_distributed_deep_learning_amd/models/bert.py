"""BERT-base / BERT-large encoder + sequence-classification head (post-LN).

Parameter-for-parameter equivalent to HF ``BertForSequenceClassification``
(109,483,778 params for base with 2 labels) except that Q, K and V are one fused
``[3·hidden, hidden]`` projection (a single MFMA GEMM writing the packed QKV the
attention kernel reads).  ``from_hf_state_dict`` / ``to_hf_state_dict`` convert
between the two naming schemes so HF checkpoints load one-to-one.

The reference's NLP half is an empty README (``notebooks/nlp/README.md``); the
workload is defined by BASELINE.json:9,11.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from ..ops.bridge import GradBridge
from .layers import Dropout, Embedding, LayerNorm, Linear


def _bridge(h: torch.Tensor):
    return GradBridge() if (torch.is_grad_enabled() and h.requires_grad) else None


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    initializer_range: float = 0.02
    num_labels: int = 2

    @classmethod
    def base(cls, **kw):
        return cls(**kw)

    @classmethod
    def large(cls, **kw):
        d = dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096)
        d.update(kw)
        return cls(**d)


class BertEmbeddings(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        std = c.initializer_range
        self.word_embeddings = Embedding(c.vocab_size, c.hidden_size, std)
        self.position_embeddings = Embedding(c.max_position_embeddings, c.hidden_size, std)
        self.token_type_embeddings = Embedding(c.type_vocab_size, c.hidden_size, std)
        self.LayerNorm = LayerNorm(c.hidden_size, c.layer_norm_eps)
        self.dropout = Dropout(c.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids=None):
        B, S = input_ids.shape
        we = self.word_embeddings(input_ids)
        if token_type_ids is None:
            # position rows + token type 0 in one native pass; its backward writes both parameters'
            # gradient slots directly (ops/glue.py)
            r = ops.embedding_residual(self.position_embeddings.weight, self.token_type_embeddings.weight, S)
        else:
            r = self.position_embeddings.weight[:S].unsqueeze(0) + self.token_type_embeddings(token_type_ids)
        h = self.LayerNorm(we, residual=r)
        return self.dropout(h)


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        H, I, std = c.hidden_size, c.intermediate_size, c.initializer_range
        self.num_heads = c.num_attention_heads
        self.attn_dropout = c.attention_probs_dropout_prob
        self.qkv = Linear(H, 3 * H, init_std=std)
        self.attn_out = Linear(H, H, init_std=std)
        self.attn_ln = LayerNorm(H, c.layer_norm_eps)
        self.ffn_in = Linear(H, I, act="gelu", init_std=std)
        self.ffn_out = Linear(I, H, init_std=std)
        self.ffn_ln = LayerNorm(H, c.layer_norm_eps)
        self.dropout = Dropout(c.hidden_dropout_prob)
        for lin in (self.qkv, self.attn_out, self.ffn_in, self.ffn_out):
            nn.init.zeros_(lin.bias)

    def forward(self, h, mask: Optional[torch.Tensor] = None):
        # hidden dropout fused into the post-LN kernels: LN(dropout(sublayer) + h); each
        # residual gradient is bridged into the dgrad epilogue of the Linear that also
        # reads h (qkv / ffn_in) instead of an autograd add
        br1, br2 = _bridge(h), None
        qkv = self.qkv(h, grad_residual=br1)
        ctx = ops.attention(qkv, self.num_heads, mask, self.attn_dropout, self.training)
        h = self.attn_ln(self.attn_out(ctx), residual=h, dropout=self.dropout.p, residual_grad_to=br1)
        br2 = _bridge(h)
        # ffn_in's GELU backward runs in ffn_out's dgrad epilogue (ffn_out is its only consumer)
        f = self.ffn_out(self.ffn_in(h, grad_residual=br2), fuse_dgelu=True)
        return self.ffn_ln(f, residual=h, dropout=self.dropout.p, residual_grad_to=br2)


class BertModel(nn.Module):
    # ZeRO-1 gather waits (parallel/ddp.py): only dispatches to its children's forwards
    _ddl_gather_router = True

    def __init__(self, c: BertConfig):
        super().__init__()
        self.config = c
        self.embeddings = BertEmbeddings(c)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.num_hidden_layers)])
        self.pooler = Linear(c.hidden_size, c.hidden_size, act="tanh", init_std=c.initializer_range)
        nn.init.zeros_(self.pooler.bias)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None):
        mask_bias = None
        if attention_mask is not None:
            mask_bias = (1.0 - attention_mask.float()) * -10000.0
        h = self.embeddings(input_ids, token_type_ids)
        for layer in self.layers:
            h = layer(h, mask_bias)
        pooled = self.pooler(ops.first_token(h))
        return h, pooled


class BertForSequenceClassification(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.config = c
        self.bert = BertModel(c)
        self.dropout = Dropout(c.hidden_dropout_prob)
        self.classifier = Linear(c.hidden_size, c.num_labels, init_std=c.initializer_range)
        nn.init.zeros_(self.classifier.bias)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None):
        _, pooled = self.bert(input_ids, attention_mask, token_type_ids)
        logits = self.classifier(self.dropout(pooled))
        if labels is not None:
            return ops.cross_entropy(logits, labels), logits
        return logits


def bert_base(num_labels: int = 2, dropout: float = 0.1, **kw) -> BertForSequenceClassification:
    return BertForSequenceClassification(BertConfig.base(num_labels=num_labels, hidden_dropout_prob=dropout,
                                                         attention_probs_dropout_prob=dropout, **kw))


def bert_large(num_labels: int = 2, dropout: float = 0.1, **kw) -> BertForSequenceClassification:
    return BertForSequenceClassification(BertConfig.large(num_labels=num_labels, hidden_dropout_prob=dropout,
                                                          attention_probs_dropout_prob=dropout, **kw))


def bert_tiny(num_labels: int = 2, dropout: float = 0.1, **kw) -> BertForSequenceClassification:
    """2 layers, hidden 128, 2 heads: the BERT code path at test / smoke size."""
    d = dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
             vocab_size=1024, max_position_embeddings=128)
    d.update(kw)
    return BertForSequenceClassification(BertConfig(num_labels=num_labels, hidden_dropout_prob=dropout,
                                                    attention_probs_dropout_prob=dropout, **d))


# ------------------------------------------------------------ HF conversion
_HF_LAYER_MAP = {
    "attention.output.dense": "attn_out",
    "attention.output.LayerNorm": "attn_ln",
    "intermediate.dense": "ffn_in",
    "output.dense": "ffn_out",
    "output.LayerNorm": "ffn_ln",
}


def from_hf_state_dict(sd: dict, num_layers: int) -> dict:
    """HF ``BertForSequenceClassification`` state dict -> this model's."""
    out = {}
    for k, v in sd.items():
        if k.startswith("bert.embeddings.") and "position_ids" not in k and "token_type_ids" not in k:
            out[k] = v
        elif k.startswith("bert.pooler.dense."):
            out[k.replace("bert.pooler.dense.", "bert.pooler.")] = v
        elif k.startswith("classifier."):
            out[k] = v
    for i in range(num_layers):
        p = f"bert.encoder.layer.{i}."
        for t in ("weight", "bias"):
            out[f"bert.layers.{i}.qkv.{t}"] = torch.cat(
                [sd[p + f"attention.self.{n}.{t}"] for n in ("query", "key", "value")], 0)
            for hf, ours in _HF_LAYER_MAP.items():
                out[f"bert.layers.{i}.{ours}.{t}"] = sd[p + f"{hf}.{t}"]
    return out


def to_hf_state_dict(sd: dict, num_layers: int) -> dict:
    out = {}
    for k, v in sd.items():
        if k.startswith("bert.embeddings.") or k.startswith("classifier."):
            out[k] = v
        elif k.startswith("bert.pooler."):
            out[k.replace("bert.pooler.", "bert.pooler.dense.")] = v
    for i in range(num_layers):
        p = f"bert.encoder.layer.{i}."
        for t in ("weight", "bias"):
            q, kk, vv = sd[f"bert.layers.{i}.qkv.{t}"].chunk(3, 0)
            out[p + f"attention.self.query.{t}"] = q
            out[p + f"attention.self.key.{t}"] = kk
            out[p + f"attention.self.value.{t}"] = vv
            for hf, ours in _HF_LAYER_MAP.items():
                out[p + f"{hf}.{t}"] = sd[f"bert.layers.{i}.{ours}.{t}"]
    return out
