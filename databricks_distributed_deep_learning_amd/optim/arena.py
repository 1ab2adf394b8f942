"""Flat parameter / gradient arena.

MI355X-first layout decision: every trainable parameter of a model lives as a
view into ONE contiguous buffer (per dtype), and every gradient as a view into a
second buffer with the identical layout.  Consequences:

* the data-parallel reducer all-reduces contiguous slices of the gradient arena
  directly (no flatten / unflatten copies, few large RCCL messages);
* the optimizer step is one fused elementwise HIP launch over the whole arena
  (``ops.optim_kernels``) instead of 161 (ResNet-50) or ~200 (BERT) per-tensor
  launches, with a per-block tensor table for per-tensor hyper-parameters
  (weight-decay masks, LAMB trust ratios);
* the layout is ordered in *reverse* registration order so the first bucket to
  fill during backward is the first one in memory.

Each tensor starts on an ``align``-element boundary so 16-byte vector loads of
bf16 and fp32 never straddle tensors.
"""
from __future__ import annotations

import weakref
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

BLOCK_ELEMS = 8192  # elements per optimizer work item (one 256-thread block)


@dataclass
class ArenaEntry:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    shape: Tuple[int, ...]
    decay: bool


def default_no_decay(name: str, p: torch.Tensor) -> bool:
    """HF/BERT convention: no weight decay on biases and normalisation weights."""
    lname = name.lower()
    return p.dim() <= 1 or lname.endswith(".bias") or "norm" in lname or "bn" in lname


class ParamArena:
    def __init__(self, named_params: Sequence[Tuple[str, nn.Parameter]], align: int = 64,
                 reverse: bool = True, no_decay_fn=default_no_decay, pad_multiple: int = 1):
        """``pad_multiple``: the flat length is rounded up to a multiple of it (a sharded
        optimizer needs ``world * align`` so every rank owns an equal, aligned slice)."""
        named_params = [(n, p) for n, p in named_params if p.requires_grad]
        if not named_params:
            raise ValueError("ParamArena: no trainable parameters")
        dtypes = {p.dtype for _, p in named_params}
        devices = {p.device for _, p in named_params}
        if len(dtypes) != 1 or len(devices) != 1:
            raise ValueError(f"ParamArena needs one dtype/device, got {dtypes} {devices}")
        self.dtype = dtypes.pop()
        self.device = devices.pop()
        order = list(reversed(named_params)) if reverse else list(named_params)
        entries: List[ArenaEntry] = []
        off = 0
        for name, p in order:
            n = p.numel()
            entries.append(ArenaEntry(name, p, off, n, tuple(p.shape), not no_decay_fn(name, p)))
            off += (n + align - 1) // align * align
        pad = max(1, int(pad_multiple))
        self.numel = (off + pad - 1) // pad * pad
        off = self.numel
        self.entries = entries
        self.flat = torch.zeros(off, dtype=self.dtype, device=self.device)
        self.grad = torch.zeros(off, dtype=self.dtype, device=self.device)
        # Bumped by every write to ``flat`` that bypasses the parameters' own version
        # counters (the flat optimizers write through raw pointers / the arena tensor,
        # whose counter is not the views'): caches derived from a weight key on it.
        self.generation = 0
        with torch.no_grad():
            for e in entries:
                view = self.flat[e.offset:e.offset + e.numel].view(e.shape)
                view.copy_(e.param.data)
                e.param.data = view
                e.param.grad = self.grad[e.offset:e.offset + e.numel].view(e.shape)
                e.param._ddl_arena = weakref.ref(self)
        self._tables: Dict[Tuple[str, int], torch.Tensor] = {}

    def bump(self) -> None:
        """Record that the parameters changed (invalidates weight-derived caches)."""
        self.generation += 1

    # ------------------------------------------------------------------
    def rebind_grads(self) -> None:
        """Re-point ``p.grad`` at the arena (after someone set grads to None)."""
        for e in self.entries:
            g = e.param.grad
            if g is None or g.data_ptr() != self.grad[e.offset:].data_ptr():
                view = self.grad[e.offset:e.offset + e.numel].view(e.shape)
                if g is not None:
                    view.copy_(g)
                e.param.grad = view

    def zero_grad(self) -> None:
        from ..ops import _lib
        if self.grad.is_cuda and _lib.mode() != "off" and _lib.available():
            from ..ops import _native_elementwise as E
            E.zero_(self.grad)          # the framework's own fill kernel (no ATen launch)
        else:
            self.grad.zero_()

    def param_views(self, flat: torch.Tensor) -> List[torch.Tensor]:
        return [flat[e.offset:e.offset + e.numel].view(e.shape) for e in self.entries]

    def block_table(self, device=None, block: int = BLOCK_ELEMS) -> torch.Tensor:
        """int32 [nblocks, 4] rows: (start, length, tensor_index, decay_flag)."""
        device = device or self.device
        key = (str(device), block)
        if key not in self._tables:
            rows = []
            for ti, e in enumerate(self.entries):
                s = 0
                while s < e.numel:
                    ln = min(block, e.numel - s)
                    rows.append((e.offset + s, ln, ti, 1 if e.decay else 0))
                    s += ln
            self._tables[key] = torch.tensor(rows, dtype=torch.int32, device=device)
        return self._tables[key]

    def tensor_table(self, device=None) -> torch.Tensor:
        """int64 [ntensors, 2] rows: (offset, numel) — segments for per-tensor norms."""
        device = device or self.device
        return torch.tensor([(e.offset, e.numel) for e in self.entries], dtype=torch.int64, device=device)

    def decay_mask(self) -> torch.Tensor:
        m = torch.zeros(self.numel, dtype=torch.bool, device=self.device)
        for e in self.entries:
            if e.decay:
                m[e.offset:e.offset + e.numel] = True
        return m

    def __len__(self) -> int:
        return len(self.entries)
