"""Synthetic, device-resident data loaders (north-star N3).

Replaces the Petastorm / Delta Lake reader named in BASELINE.json:5.  Batches
are generated once, directly on the rank's device, with per-rank seeds (so
ranks see different data, as a rank-sharded real loader would), and cycled —
no host->device copy and no host work in the training hot loop.

Image batches are NHWC, pre-normalised with the ImageNet mean/std the reference
uses (``notebooks/cv/onnx_experiments.py:63``), labels uniform in
[0, num_classes).  Token batches are ids uniform in [0, vocab) with an
all-ones attention mask by default (optionally random right-padding).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _gen(device, seed: int) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


class SyntheticImageNet:
    def __init__(self, batch_size: int, image_size: int = 224, num_classes: int = 1000,
                 device: Optional[torch.device] = None, dtype: torch.dtype = torch.float32,
                 rank: int = 0, seed: int = 1234, pool: int = 4, steps_per_epoch: int = 0,
                 channels_last: bool = True):
        self.batch_size, self.image_size, self.num_classes = batch_size, image_size, num_classes
        self.device = device or torch.device("cpu")
        self.dtype = dtype
        self.steps_per_epoch = steps_per_epoch
        g = _gen(self.device, seed * 1000 + rank)
        shape = (batch_size, image_size, image_size, 3) if channels_last else (batch_size, 3, image_size, image_size)
        self.pool = []
        for _ in range(max(1, pool)):
            x = torch.randn(shape, generator=g, device=self.device, dtype=torch.float32)
            x = x.to(dtype)
            y = torch.randint(0, num_classes, (batch_size,), generator=g, device=self.device)
            self.pool.append((x, y))
        self._i = 0

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        n = 0
        while self.steps_per_epoch <= 0 or n < self.steps_per_epoch:
            yield self.next()
            n += 1

    def next(self) -> Tuple[torch.Tensor, torch.Tensor]:
        b = self.pool[self._i % len(self.pool)]
        self._i += 1
        return b

    def __len__(self):
        return self.steps_per_epoch

    def state_dict(self):
        """Loader position (checkpoint / resume replays the same batch sequence)."""
        return {"index": self._i}

    def load_state_dict(self, st) -> None:
        self._i = int(st["index"])


class SyntheticTokens:
    def __init__(self, batch_size: int, seq_len: int = 128, vocab_size: int = 30522, num_labels: int = 2,
                 device: Optional[torch.device] = None, rank: int = 0, seed: int = 1234, pool: int = 4,
                 pad_fraction: float = 0.0, steps_per_epoch: int = 0):
        self.batch_size, self.seq_len = batch_size, seq_len
        self.device = device or torch.device("cpu")
        self.steps_per_epoch = steps_per_epoch
        g = _gen(self.device, seed * 1000 + rank + 7)
        self.pool = []
        for _ in range(max(1, pool)):
            ids = torch.randint(0, vocab_size, (batch_size, seq_len), generator=g, device=self.device)
            mask = None
            if pad_fraction > 0:
                lens = torch.randint(int(seq_len * (1 - pad_fraction)), seq_len + 1, (batch_size,),
                                     generator=g, device=self.device)
                mask = (torch.arange(seq_len, device=self.device)[None, :] < lens[:, None]).to(torch.int64)
            labels = torch.randint(0, num_labels, (batch_size,), generator=g, device=self.device)
            self.pool.append({"input_ids": ids, "attention_mask": mask, "labels": labels})
        self._i = 0

    def __iter__(self):
        n = 0
        while self.steps_per_epoch <= 0 or n < self.steps_per_epoch:
            yield self.next()
            n += 1

    def next(self):
        b = self.pool[self._i % len(self.pool)]
        self._i += 1
        return b

    def __len__(self):
        return self.steps_per_epoch

    def state_dict(self):
        """Loader position (checkpoint / resume replays the same batch sequence)."""
        return {"index": self._i}

    def load_state_dict(self, st) -> None:
        self._i = int(st["index"])


def shard_indices(n: int, rank: int, world: int, shuffle: bool = False, seed: int = 0, drop_last: bool = True):
    """Rank-sharded index list (what a DistributedSampler yields) for real datasets."""
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(seed)) if shuffle else torch.arange(n)
    per = n // world if drop_last else -(-n // world)
    if not drop_last:
        idx = torch.cat([idx, idx[: per * world - n]])
    return idx[rank * per:(rank + 1) * per].tolist()
