"""Dataclass configuration + presets for the five north-star workloads.

The reference hard-codes every constant in the notebook (image size at
``notebooks/cv/onnx_experiments.py:29-30``, opset at :38, ``/tmp`` paths at
:36,48,81,198,215).  Here every knob lives in one dataclass that can be
overridden from the CLI (``--key=value``) or the environment (``DDL_KEY=value``).
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional


@dataclass
class TrainConfig:
    # ---- workload ---------------------------------------------------------
    model: str = "resnet50"          # resnet18|resnet34|resnet50|resnet101|bert_base|bert_large|vit_b16|...
    task: str = "auto"               # auto|cv|nlp
    num_classes: int = 1000          # CV classes / NLP labels (num_labels)
    image_size: int = 224
    seq_len: int = 128
    vocab_size: int = 30522
    batch_size: int = 256            # per-rank micro-batch
    grad_accum: int = 1              # micro-steps per optimizer step
    steps: int = 50                  # optimizer steps to run
    warmup_steps: int = 5            # untimed optimizer steps
    epochs: int = 1
    # ---- numerics ---------------------------------------------------------
    dtype: str = "bf16"              # bf16|fp32 compute dtype (master weights are fp32)
    dropout: float = 0.1             # NLP hidden/attention dropout (0 disables)
    # ---- optimizer --------------------------------------------------------
    optimizer: str = "auto"          # auto|sgd|adamw|lamb
    lr: float = 0.1
    momentum: float = 0.9
    nesterov: bool = False
    weight_decay: float = 5e-5
    betas: List[float] = field(default_factory=lambda: [0.9, 0.999])
    eps: float = 1e-6
    max_grad_norm: float = 0.0       # 0 disables global-norm clipping
    lr_schedule: str = "constant"    # constant|linear|cosine
    lr_warmup_steps: int = 0
    # ---- distributed ------------------------------------------------------
    backend: str = "auto"            # auto|nccl|gloo  (nccl == RCCL on ROCm)
    bucket_mb: float = 0.0           # gradient bucket size for the reducer (<= 0: "auto" -- sized from the
                                     # startup all-reduce probe at world > 1 with the native engine; the
                                     # 4 / 25 MB constants without a probe; bucket_policy.source says which)
    first_bucket_mb: float = 4.0     # small first bucket so comm starts early (fixed bucket_mb only)
    comm_probe: bool = False         # probe even with a fixed bucket_mb (the auto policy always probes)
    comm: str = "auto"               # gradient all-reduce engine: auto|native (C++ RCCL engine)|torch
    grad_reduce_dtype: str = "auto"  # auto|fp32|bf16  all-reduce payload dtype
    broadcast_buffers: bool = False
    sync_bn: bool = False            # SyncBatchNorm: BN statistics summed over all ranks (CV models)
    zero_optimizer: bool = False     # ZeRO-1: fp32 master + optimizer state sharded 1/world per rank
    overlap_optimizer: bool = True   # world > 1: per-bucket optimizer updates as each all-reduce completes
    dp_rehearsal: bool = False       # world 1 on a GPU: run the N > 1 step's form anyway -- native RCCL
                                     # engine (1-rank communicator), per-bucket all-reduces, per-bucket
                                     # range optimizer (overlap_optimizer) -- so its cost shows in phases_ms
    eager_optimizer: bool = False    # GPU: those updates start during backward, on a side stream
                                     # (1 GPU same-box A/B: -0.4 % -- the HBM-bound updates slow the
                                     # concurrent backward GEMMs about as much as they hide)
    # ---- runtime ----------------------------------------------------------
    native: str = "auto"             # auto|on|off  HIP kernels (off = stock torch ops)
    seed: int = 1234
    log_every: int = 10
    log_file: str = ""               # JSONL metrics (rank 0)
    phase_timing: bool = True        # fwd/bwd/comm_wait/opt HIP-event breakdown in the log + summary
    checkpoint_dir: str = ""
    checkpoint_every: int = 0
    resume: bool = False
    fault_rank: int = -1             # test-only fault injection (rank that raises)
    fault_step: int = -1
    check_replicas_every: int = 0    # debug: every N steps assert DP replicas hold identical params
    data: str = "synthetic"          # synthetic (Petastorm/Delta replacement)
    synthetic_pool: int = 4          # distinct device-resident batches cycled
    pad_fraction: float = 0.0        # NLP: random right-padding up to this fraction (attention-mask path)

    # ---------------------------------------------------------------------
    @property
    def resolved_task(self) -> str:
        if self.task != "auto":
            return self.task
        return "nlp" if self.model.startswith("bert") else "cv"

    @property
    def resolved_optimizer(self) -> str:
        if self.optimizer != "auto":
            return self.optimizer
        if self.model.startswith("bert_large"):
            return "lamb"
        if self.model.startswith(("bert", "vit")):
            return "adamw"
        return "sgd"

    def replace(self, **kw) -> "TrainConfig":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "TrainConfig":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})


def _coerce(value: str, proto: Any) -> Any:
    if isinstance(proto, bool):
        return value.lower() in ("1", "true", "yes", "on")
    if isinstance(proto, int):
        return int(value)
    if isinstance(proto, float):
        return float(value)
    if isinstance(proto, list):
        return [float(v) for v in value.split(",")]
    return value


def apply_overrides(cfg: TrainConfig, argv: Optional[List[str]] = None,
                    env: Optional[Dict[str, str]] = None) -> TrainConfig:
    """Apply ``DDL_<KEY>`` env vars, then ``--key=value`` / ``--key value`` args."""
    env = os.environ if env is None else env
    kw: Dict[str, Any] = {}
    protos = {f.name: getattr(cfg, f.name) for f in fields(cfg)}
    for name, proto in protos.items():
        ev = env.get("DDL_" + name.upper())
        if ev is not None:
            kw[name] = _coerce(ev, proto)
    argv = list(argv or [])
    i = 0
    while i < len(argv):
        a = argv[i]
        if a.startswith("--"):
            key, _, val = a[2:].partition("=")
            key = key.replace("-", "_")
            if key in protos:
                if val == "" and "=" not in a:
                    if isinstance(protos[key], bool) and (i + 1 >= len(argv) or argv[i + 1].startswith("--")):
                        val = "true"
                    else:
                        i += 1
                        val = argv[i]
                kw[key] = _coerce(val, protos[key])
        i += 1
    return cfg.replace(**kw)


# The five configurations named by BASELINE.json:7-11.
PRESETS: Dict[str, TrainConfig] = {
    # BJ:7 — plumbing slice, CPU / gloo, world_size=2
    "resnet18_gloo": TrainConfig(model="resnet18", batch_size=8, image_size=224, steps=3,
                                 warmup_steps=1, dtype="fp32", backend="gloo", native="off",
                                 lr=0.1),
    # BJ:8 — ResNet-50 bf16 DDP, synthetic ImageNet-shape batches
    "resnet50_ddp": TrainConfig(model="resnet50", batch_size=256, dtype="bf16", optimizer="sgd",
                                lr=0.1, weight_decay=5e-5),
    # BJ:9 — BERT-base fine-tune seq 128 (HF-style loop)
    "bert_base_ddp": TrainConfig(model="bert_base", batch_size=128, seq_len=128, num_classes=2,
                                 dtype="bf16", optimizer="adamw", lr=2e-5, weight_decay=0.01,
                                 eps=1e-6, dropout=0.1),
    # BJ:10 — ViT-B/16 bf16 (shares NLP kernels)
    "vit_b16": TrainConfig(model="vit_b16", batch_size=128, dtype="bf16", optimizer="adamw",
                           lr=1e-3, weight_decay=0.05, dropout=0.0),
    # BJ:11 — BERT-large s512 + LAMB + grad-accum + HBM-aware batch sizing
    "bert_large_lamb": TrainConfig(model="bert_large", batch_size=0, seq_len=512, num_classes=2,
                                   grad_accum=4, dtype="bf16", optimizer="lamb", lr=2e-3,
                                   weight_decay=0.01, dropout=0.1),
}


def get_preset(name: str, **overrides) -> TrainConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; have {sorted(PRESETS)}")
    return PRESETS[name].replace(**overrides)
