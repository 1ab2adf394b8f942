"""Flat-arena optimizers with fp32 master weights (N12; kernels K12/K20/K21/K22).

All state (fp32 master copy, momentum / Adam moments) is stored flat with the
arena's layout, so one optimizer step is ONE fused HIP kernel over the arena
(``csrc/kernels/optim.hip``) reading bf16 (or fp32) gradients, updating the
fp32 master and writing the bf16 compute copy in the same pass.  LAMB adds one
segmented-norm kernel for the per-tensor trust ratios.  On CPU the same math
runs as vectorised torch ops on the flat tensors.

Update rules follow the PyTorch definitions (SGD with coupled weight decay,
AdamW with decoupled decay) and the LAMB paper (You et al. 2019, trust ratio
||p|| / ||update|| per tensor, bias-corrected moments).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

from .arena import ParamArena
from ..ops import _lib


class FlatOptimizer:
    name = "base"

    def __init__(self, arena: ParamArena, lr: float, weight_decay: float = 0.0,
                 max_grad_norm: float = 0.0):
        self.arena = arena
        self.lr = lr
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self.master: Optional[torch.Tensor] = None
        if arena.dtype != torch.float32:
            self.master = arena.flat.detach().float().clone()
        self._decay_mask: Optional[torch.Tensor] = None
        self.last_grad_norm: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------
    @property
    def params32(self) -> torch.Tensor:
        return self.master if self.master is not None else self.arena.flat

    def decay_mask(self) -> torch.Tensor:
        if self._decay_mask is None:
            self._decay_mask = self.arena.decay_mask().to(torch.float32)
        return self._decay_mask

    def _native(self) -> bool:
        return _lib.use_native(self.arena.flat)

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.arena.zero_grad()

    def _clip_scale(self, grad: torch.Tensor, grad_scale: float) -> torch.Tensor:
        """Returns a device scalar multiplier (grad_scale, times the clip factor)."""
        if self.max_grad_norm and self.max_grad_norm > 0:
            if self._native():
                from ..ops import _native_optim
                norm = _native_optim.global_norm(grad) * grad_scale
            else:
                norm = grad.float().norm() * grad_scale
            self.last_grad_norm = norm
            clip = torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
            return clip * grad_scale
        return torch.full((), grad_scale, dtype=torch.float32, device=grad.device)

    @torch.no_grad()
    def step(self, grad: Optional[torch.Tensor] = None, grad_scale: float = 1.0, lr: Optional[float] = None):
        if grad is None:
            grad = self.arena.grad
        self.step_count += 1
        if lr is not None:
            self.lr = lr
        scale = self._clip_scale(grad, grad_scale)
        if self._native():
            self._step_native(grad, scale)
        else:
            self._step_torch(grad.float() * scale)
            if self.master is not None:
                self.arena.flat.copy_(self.master)

    # ------------------------------------------------------------------
    def state_dict(self) -> Dict[str, object]:
        st = {"name": self.name, "step": self.step_count, "lr": self.lr}
        if self.master is not None:
            st["master"] = self.master
        st.update(self._state_tensors())
        return st

    def load_state_dict(self, st: Dict[str, object]) -> None:
        self.step_count = int(st["step"])
        self.lr = float(st["lr"])
        if self.master is not None and "master" in st:
            self.master.copy_(st["master"])
            self.arena.flat.copy_(self.master)
        for k, t in self._state_tensors().items():
            t.copy_(st[k])

    def _state_tensors(self) -> Dict[str, torch.Tensor]:
        return {}


class FlatSGD(FlatOptimizer):
    name = "sgd"

    def __init__(self, arena, lr=0.1, momentum=0.9, weight_decay=0.0, nesterov=False, max_grad_norm=0.0):
        super().__init__(arena, lr, weight_decay, max_grad_norm)
        self.momentum, self.nesterov = momentum, nesterov
        self.buf = torch.zeros(arena.numel, dtype=torch.float32, device=arena.device)

    def _state_tensors(self):
        return {"momentum_buffer": self.buf}

    def _step_torch(self, g):
        p = self.params32
        d = g + self.weight_decay * self.decay_mask() * p if self.weight_decay else g
        if self.momentum:
            if self.step_count == 1:
                self.buf.copy_(d)
            else:
                self.buf.mul_(self.momentum).add_(d)
            d = d + self.momentum * self.buf if self.nesterov else self.buf
        p.add_(d, alpha=-self.lr)

    def _step_native(self, grad, scale):
        from ..ops import _native_optim
        _native_optim.sgd(self, grad, scale)


class FlatAdamW(FlatOptimizer):
    name = "adamw"

    def __init__(self, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=0.0):
        super().__init__(arena, lr, weight_decay, max_grad_norm)
        self.b1, self.b2 = betas
        self.eps = eps
        self.m = torch.zeros(arena.numel, dtype=torch.float32, device=arena.device)
        self.v = torch.zeros(arena.numel, dtype=torch.float32, device=arena.device)

    def _state_tensors(self):
        return {"exp_avg": self.m, "exp_avg_sq": self.v}

    def _step_torch(self, g):
        p = self.params32
        t = self.step_count
        if self.weight_decay:
            p.mul_(1.0 - self.lr * self.weight_decay * self.decay_mask())
        self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        bc1 = 1 - self.b1 ** t
        bc2 = 1 - self.b2 ** t
        denom = (self.v / bc2).sqrt_().add_(self.eps)
        p.addcdiv_(self.m, denom, value=-self.lr / bc1)

    def _step_native(self, grad, scale):
        from ..ops import _native_optim
        _native_optim.adamw(self, grad, scale)


class FlatLAMB(FlatOptimizer):
    name = "lamb"

    def __init__(self, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_grad_norm=1.0,
                 bias_correction=True):
        super().__init__(arena, lr, weight_decay, max_grad_norm)
        self.b1, self.b2 = betas
        self.eps = eps
        self.bias_correction = bias_correction
        self.m = torch.zeros(arena.numel, dtype=torch.float32, device=arena.device)
        self.v = torch.zeros(arena.numel, dtype=torch.float32, device=arena.device)
        self.u = torch.empty(0)  # scratch for the torch path

    def _state_tensors(self):
        return {"exp_avg": self.m, "exp_avg_sq": self.v}

    def _step_torch(self, g):
        p = self.params32
        t = self.step_count
        self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        bc1 = 1 - self.b1 ** t if self.bias_correction else 1.0
        bc2 = 1 - self.b2 ** t if self.bias_correction else 1.0
        u = (self.m / bc1) / ((self.v / bc2).sqrt() + self.eps)
        if self.weight_decay:
            u = u + self.weight_decay * self.decay_mask() * p
        for e in self.arena.entries:
            sl = slice(e.offset, e.offset + e.numel)
            pn = p[sl].norm()
            un = u[sl].norm()
            ratio = torch.where((pn > 0) & (un > 0), pn / un, torch.ones_like(pn))
            p[sl].add_(u[sl] * ratio, alpha=-self.lr)

    def _step_native(self, grad, scale):
        from ..ops import _native_optim
        _native_optim.lamb(self, grad, scale)


def build_optimizer(name: str, arena: ParamArena, cfg) -> FlatOptimizer:
    if name == "sgd":
        return FlatSGD(arena, lr=cfg.lr, momentum=cfg.momentum, weight_decay=cfg.weight_decay,
                       nesterov=cfg.nesterov, max_grad_norm=cfg.max_grad_norm)
    if name == "adamw":
        return FlatAdamW(arena, lr=cfg.lr, betas=tuple(cfg.betas), eps=cfg.eps, weight_decay=cfg.weight_decay,
                         max_grad_norm=cfg.max_grad_norm)
    if name == "lamb":
        return FlatLAMB(arena, lr=cfg.lr, betas=tuple(cfg.betas), eps=cfg.eps, weight_decay=cfg.weight_decay,
                        max_grad_norm=cfg.max_grad_norm or 1.0)
    raise KeyError(name)


class LRSchedule:
    """constant | linear (warmup then linear decay to 0) | cosine."""

    def __init__(self, base_lr: float, kind: str = "constant", warmup: int = 0, total: int = 1):
        self.base_lr, self.kind, self.warmup, self.total = base_lr, kind, warmup, max(1, total)

    def __call__(self, step: int) -> float:
        if self.warmup and step < self.warmup:
            return self.base_lr * (step + 1) / self.warmup
        if self.kind == "constant":
            return self.base_lr
        frac = min(1.0, (step - self.warmup) / max(1, self.total - self.warmup))
        if self.kind == "linear":
            return self.base_lr * (1.0 - frac)
        if self.kind == "cosine":
            return self.base_lr * 0.5 * (1.0 + math.cos(math.pi * frac))
        raise ValueError(self.kind)
