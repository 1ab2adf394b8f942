"""MI355X-native distributed deep-learning harness.

Capabilities of ``rafaelvp-db/databricks-distributed-deep-learning`` re-designed for
single-node AMD Instinct MI355X (gfx950 / CDNA4):

* ``parallel``  - process-group bootstrap, TorchDistributor / HorovodRunner style
  launchers, a bucketed data-parallel gradient reducer over RCCL (xGMI).
* ``ops``       - hand-written HIP kernels (MFMA GEMM / implicit-GEMM conv, fused
  BatchNorm+ReLU, LayerNorm, GELU, flash attention, fused optimizers) with
  autograd bindings and plain-PyTorch CPU references.
* ``models``    - ResNet-18/50, BERT-base/large, ViT-B/16 written from scratch.
* ``optim``     - flat-arena SGD / AdamW / LAMB with fp32 master weights.
* ``data``      - synthetic ImageNet / token loaders (replace Petastorm / Delta).
* ``train``     - notebook-style ``train(cfg)`` for CV and NLP.
* ``export``    - reference-parity export + inference runtime comparison
  (reference: ``notebooks/cv/onnx_experiments.py``).
"""

__version__ = "0.1.0"

from . import config  # noqa: F401
from .config import TrainConfig, PRESETS, get_preset  # noqa: F401


def train(cfg=None, **overrides):
    """Notebook-style entry point (lazy import keeps ``import`` cheap)."""
    from .training.loop import train as _train
    return _train(cfg, **overrides)
