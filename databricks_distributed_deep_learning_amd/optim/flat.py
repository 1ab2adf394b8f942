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


def _sum_over_ranks(t: torch.Tensor) -> None:
    """In-place SUM over the data-parallel ranks: through the reducer's native RCCL engine
    when one is active (one communicator for every collective of a step), else torch."""
    from ..parallel import comm as _comm
    eng = _comm.active()
    if eng is not None and t.is_cuda:
        eng.wait_upto(eng.all_reduce(t))
        return
    import torch.distributed as dist
    dist.all_reduce(t)


class FlatOptimizer:
    """``shard`` -- ZeRO-1: this rank keeps the fp32 master copy and the optimizer state
    only for the arena ranges it owns, stored back to back in a LOCAL index space.

    * ``shard=(rank, world)``: one contiguous 1/world slice of the arena (padded to
      ``world * 64`` elements);
    * ``shard=(rank, world, groups)``: ``groups`` = ``[(start, end), ...]`` gradient
      buckets (``DataParallel(shard=True).buckets``, each a multiple of ``world * 64``
      elements); the rank owns chunk ``rank`` of every bucket -- exactly what a per-bucket
      reduce-scatter leaves it, so the reduced gradient shard IS the local gradient.

    ``step(grad)`` takes the local gradient shard (or a full-arena gradient, whose owned
    pieces are gathered), updates the owned elements, writes their compute-dtype copy
    into the arena and all-gathers every group's chunks back into ``arena.flat`` -- through
    ``gather_fn`` when set (the reducer's async, stream-ordered all-gathers that the next
    forward waits on bucket by bucket), synchronously otherwise.  The kernels' block
    table carries, per row, the offset from local index to arena index, so one launch
    still covers every owned range."""
    name = "base"

    def __init__(self, arena: ParamArena, lr: float, weight_decay: float = 0.0,
                 max_grad_norm: float = 0.0, shard=None):
        self.arena = arena
        self.lr = lr
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self._scale_cache = {}
        self.shard = None
        # ranges: (arena lo, arena hi, local offset); groups: (start, end) gathered per rank chunk
        self.ranges = [(0, arena.numel, 0)]
        self.groups = []
        self.gather_fn = None
        if shard is not None and shard[1] > 1:
            rank, world = shard[0], shard[1]
            groups = list(shard[2]) if len(shard) > 2 else [(0, arena.numel)]
            ranges, off = [], 0
            for a, b in groups:
                if (b - a) % (world * 64):
                    raise ValueError("sharded optimizer: every group must be a multiple of world * 64 elements "
                                     "(build the arena with pad_multiple = world * 64)")
                n = (b - a) // world
                ranges.append((a + rank * n, a + (rank + 1) * n, off))
                off += n
            self.shard = (rank, world)
            self.ranges, self.groups = ranges, groups
        self.local_numel = sum(hi - lo for lo, hi, _ in self.ranges)
        self.master: Optional[torch.Tensor] = None
        if arena.dtype != torch.float32 or self.shard is not None:
            self.master = self._local(arena.flat).detach().float().clone()
        self._decay_mask: Optional[torch.Tensor] = None
        self.last_grad_norm: Optional[torch.Tensor] = None

    @property
    def lo(self) -> int:          # first owned arena index (the whole arena when unsharded)
        return self.ranges[0][0]

    @property
    def hi(self) -> int:
        return self.ranges[-1][1]

    @property
    def state_numel(self) -> int:
        """Elements of optimizer state this rank holds (the whole arena unless sharded)."""
        return self.local_numel

    def _local(self, full: torch.Tensor) -> torch.Tensor:
        """The owned pieces of a full-arena tensor, back to back (a view when unsharded)."""
        if self.shard is None:
            return full
        return torch.cat([full[lo:hi] for lo, hi, _ in self.ranges])

    def _scatter_local(self, local: torch.Tensor, full: torch.Tensor) -> None:
        for lo, hi, off in self.ranges:
            full[lo:hi].copy_(local[off:off + hi - lo])

    def _zeros_state(self) -> torch.Tensor:
        return torch.zeros(self.state_numel, dtype=torch.float32, device=self.arena.device)

    # ------------------------------------------------------------------
    @property
    def params32(self) -> torch.Tensor:
        return self.master if self.master is not None else self.arena.flat

    def decay_mask(self) -> torch.Tensor:
        if self._decay_mask is None:
            self._decay_mask = self._local(self.arena.decay_mask().to(torch.float32))
        return self._decay_mask

    def local_grad(self, grad: torch.Tensor) -> torch.Tensor:
        """The gradient in local index space (``grad`` is either already the shard or the
        full arena gradient)."""
        if self.shard is None or grad.numel() == self.local_numel:
            return grad
        return self._local(grad)

    def _all_gather_params(self) -> None:
        """Every rank's updated chunks -> the full compute-dtype arena (in place)."""
        if self.gather_fn is not None:
            self.gather_fn(self.groups, self.ranges)
            return
        import torch.distributed as dist
        flat = self.arena.flat
        for (a, b), (lo, hi, _) in zip(self.groups, self.ranges):
            dist.all_gather_into_tensor(flat[a:b], flat[lo:hi].clone() if not flat.is_cuda else flat[lo:hi])

    def _native(self) -> bool:
        return _lib.use_native(self.arena.flat)

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.arena.zero_grad()

    def _clip_scale(self, grad: torch.Tensor, grad_scale: float) -> torch.Tensor:
        """Returns a device scalar multiplier (grad_scale, times the clip factor)."""
        if self.max_grad_norm and self.max_grad_norm > 0:
            if self.shard is not None:
                # the local shard: sum of squares over ranks, then the root
                sq = (grad.float().pow(2).sum()).reshape(1)
                _sum_over_ranks(sq)
                norm = sq.sqrt().reshape(()) * grad_scale
            elif self._native():
                from ..ops import _native_optim
                norm = _native_optim.global_norm(grad) * grad_scale
            else:
                norm = grad.float().norm() * grad_scale
            self.last_grad_norm = norm
            clip = torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
            return clip * grad_scale
        key = (float(grad_scale), grad.device)
        t = self._scale_cache.get(key)
        if t is None:                      # one device scalar per (scale, device): no fill per step
            t = self._scale_cache[key] = torch.full((), grad_scale, dtype=torch.float32, device=grad.device)
        return t

    # ------------------------------------------------------------------ range steps
    # The data-parallel reducer can hand the optimizer one bucket (a contiguous range of
    # whole tensors) at a time, as each bucket's all-reduce completes: begin_step(),
    # step_range() per bucket, end_step() is the same update as one step() when no
    # global quantity (clip norm) couples the ranges and the state is not sharded.
    def supports_ranges(self) -> bool:
        return self.shard is None and not (self.max_grad_norm and self.max_grad_norm > 0)

    def begin_step(self, lr: Optional[float] = None) -> None:
        if not self.supports_ranges():
            raise RuntimeError(f"{self.name}: range steps need an unsharded optimizer without gradient clipping")
        self.step_count += 1
        if lr is not None:
            self.lr = lr
        self._range_scratch: Dict[str, object] = {}

    @torch.no_grad()
    def step_range(self, grad: torch.Tensor, grad_scale: float, lo: int, hi: int) -> None:
        """Update arena elements [lo, hi) (tensor-aligned) from the full-arena ``grad``."""
        if hi <= lo:
            return
        if self._native():
            s = self._range_scratch.get("scale")
            if s is None:     # one device scalar per step, not one allocation + fill per bucket
                s = self._range_scratch["scale"] = torch.full((1,), float(grad_scale), dtype=torch.float32,
                                                              device=grad.device)
            self._step_native(grad, s, (lo, hi))
        else:
            self._step_torch(grad[lo:hi].float() * grad_scale, lo, hi)
            if self.master is not None:
                self.arena.flat[lo:hi].copy_(self.master[lo:hi])

    def end_step(self) -> None:
        self._range_scratch = {}
        self.arena.bump()

    @torch.no_grad()
    def step(self, grad: Optional[torch.Tensor] = None, grad_scale: float = 1.0, lr: Optional[float] = None):
        if grad is None:
            grad = self.arena.grad
        grad = self.local_grad(grad)
        self.step_count += 1
        if lr is not None:
            self.lr = lr
        scale = self._clip_scale(grad, grad_scale)
        if self._native():
            self._step_native(grad, scale)
        else:
            self._step_torch(grad.float() * scale)
            if self.master is not None:
                if self.shard is None:
                    self.arena.flat.copy_(self.master)
                else:
                    self._scatter_local(self.master, self.arena.flat)
        if self.shard is not None:
            self._all_gather_params()
        self.arena.bump()

    # ------------------------------------------------------------------
    def _full(self, t: torch.Tensor) -> torch.Tensor:
        """A sharded (local) state tensor gathered to the whole arena (checkpoints stay
        independent of the world size and of the bucket layout)."""
        if self.shard is None:
            return t
        import torch.distributed as dist
        out = torch.zeros(self.arena.numel, dtype=t.dtype, device=t.device)
        for (a, b), (lo, hi, off) in zip(self.groups, self.ranges):
            dist.all_gather_into_tensor(out[a:b], t[off:off + hi - lo].contiguous())
        return out

    def state_dict(self) -> Dict[str, object]:
        """Full-arena tensors on every rank (sharded state is all-gathered: collective)."""
        st = {"name": self.name, "step": self.step_count, "lr": self.lr}
        if self.master is not None:
            st["master"] = self._full(self.master)
        st.update({k: self._full(v) for k, v in self._state_tensors().items()})
        return st

    def _fit(self, t: torch.Tensor) -> torch.Tensor:
        """A full-arena tensor from a checkpoint, resized to this arena (the padding
        differs between world sizes when the optimizer is sharded)."""
        n = self.arena.numel
        if t.numel() == n:
            return t
        out = torch.zeros(n, dtype=t.dtype, device=t.device)
        k = min(n, t.numel())
        out[:k] = t[:k]
        return out

    def load_state_dict(self, st: Dict[str, object]) -> None:
        self.step_count = int(st["step"])
        self.lr = float(st["lr"])
        if self.master is not None and "master" in st:
            full = self._fit(st["master"])
            self.master.copy_(self._local(full))
            self.arena.flat.copy_(full.to(self.arena.flat.dtype))
        for k, t in self._state_tensors().items():
            t.copy_(self._local(self._fit(st[k])))
        self.arena.bump()

    def _state_tensors(self) -> Dict[str, torch.Tensor]:
        return {}


class FlatSGD(FlatOptimizer):
    name = "sgd"

    def __init__(self, arena, lr=0.1, momentum=0.9, weight_decay=0.0, nesterov=False, max_grad_norm=0.0,
                 shard=None):
        super().__init__(arena, lr, weight_decay, max_grad_norm, shard)
        self.momentum, self.nesterov = momentum, nesterov
        self.buf = self._zeros_state()

    def _state_tensors(self):
        return {"momentum_buffer": self.buf}

    def _step_torch(self, g, a=0, b=None):
        """``g``: the gradient of local elements [a, b) (the whole local range by default)."""
        b = self.state_numel if b is None else b
        p = self.params32[a:b]
        buf = self.buf[a:b]
        d = g + self.weight_decay * self.decay_mask()[a:b] * p if self.weight_decay else g
        if self.momentum:
            if self.step_count == 1:
                buf.copy_(d)
            else:
                buf.mul_(self.momentum).add_(d)
            d = d + self.momentum * buf if self.nesterov else buf
        p.add_(d, alpha=-self.lr)

    def _step_native(self, grad, scale, rng=None):
        from ..ops import _native_optim
        _native_optim.sgd(self, grad, scale, rng)


class FlatAdamW(FlatOptimizer):
    name = "adamw"

    def __init__(self, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=0.0,
                 shard=None):
        super().__init__(arena, lr, weight_decay, max_grad_norm, shard)
        self.b1, self.b2 = betas
        self.eps = eps
        self.m = self._zeros_state()
        self.v = self._zeros_state()

    def _state_tensors(self):
        return {"exp_avg": self.m, "exp_avg_sq": self.v}

    def _step_torch(self, g, a=0, b=None):
        b = self.state_numel if b is None else b
        p, m, v = self.params32[a:b], self.m[a:b], self.v[a:b]
        t = self.step_count
        if self.weight_decay:
            p.mul_(1.0 - self.lr * self.weight_decay * self.decay_mask()[a:b])
        m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        bc1 = 1 - self.b1 ** t
        bc2 = 1 - self.b2 ** t
        denom = (v / bc2).sqrt_().add_(self.eps)
        p.addcdiv_(m, denom, value=-self.lr / bc1)

    def _step_native(self, grad, scale, rng=None):
        from ..ops import _native_optim
        _native_optim.adamw(self, grad, scale, rng)


class FlatLAMB(FlatOptimizer):
    name = "lamb"

    def __init__(self, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_grad_norm=1.0,
                 bias_correction=True, shard=None):
        super().__init__(arena, lr, weight_decay, max_grad_norm, shard)
        self.b1, self.b2 = betas
        self.eps = eps
        self.bias_correction = bias_correction
        self.m = self._zeros_state()
        self.v = self._zeros_state()
        self.u = torch.empty(0)  # scratch for the torch path

    def _state_tensors(self):
        return {"exp_avg": self.m, "exp_avg_sq": self.v}

    def _step_torch(self, g, ra=0, rb=None):
        rb = self.state_numel if rb is None else rb
        p, m, v = self.params32[ra:rb], self.m[ra:rb], self.v[ra:rb]
        t = self.step_count
        m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        bc1 = 1 - self.b1 ** t if self.bias_correction else 1.0
        bc2 = 1 - self.b2 ** t if self.bias_correction else 1.0
        u = (m / bc1) / ((v / bc2).sqrt() + self.eps)
        if self.weight_decay:
            u = u + self.weight_decay * self.decay_mask()[ra:rb] * p
        # per-tensor ||p||^2, ||u||^2 over this rank's pieces of each tensor (summed over ranks when
        # sharded), restricted to local range [ra, rb); segment offsets relative to ra
        segs = [[] for _ in self.arena.entries]
        for ti, e in enumerate(self.arena.entries):
            for lo, hi, off in self.ranges:
                a, b = max(e.offset, lo), min(e.offset + e.numel, hi)
                if a < b:
                    la, lb = max(a - lo + off, ra), min(b - lo + off, rb)
                    if la < lb:
                        segs[ti].append((la - ra, lb - ra))
        sq = torch.zeros(2 * len(segs), dtype=torch.float32, device=p.device)
        for ti, sg in enumerate(segs):
            for a, b in sg:
                sq[2 * ti] += p[a:b].pow(2).sum()
                sq[2 * ti + 1] += u[a:b].pow(2).sum()
        if self.shard is not None:
            _sum_over_ranks(sq)
        for ti, sg in enumerate(segs):
            if not sg:
                continue
            pn, un = sq[2 * ti].sqrt(), sq[2 * ti + 1].sqrt()
            ratio = torch.where((pn > 0) & (un > 0), pn / un, torch.ones_like(pn))
            for a, b in sg:
                p[a:b].add_(u[a:b] * ratio, alpha=-self.lr)

    def _step_native(self, grad, scale, rng=None):
        from ..ops import _native_optim
        _native_optim.lamb(self, grad, scale, rng)


def build_optimizer(name: str, arena: ParamArena, cfg, shard=None) -> FlatOptimizer:
    if name == "sgd":
        return FlatSGD(arena, lr=cfg.lr, momentum=cfg.momentum, weight_decay=cfg.weight_decay,
                       nesterov=cfg.nesterov, max_grad_norm=cfg.max_grad_norm, shard=shard)
    if name == "adamw":
        return FlatAdamW(arena, lr=cfg.lr, betas=tuple(cfg.betas), eps=cfg.eps, weight_decay=cfg.weight_decay,
                         max_grad_norm=cfg.max_grad_norm, shard=shard)
    if name == "lamb":
        return FlatLAMB(arena, lr=cfg.lr, betas=tuple(cfg.betas), eps=cfg.eps, weight_decay=cfg.weight_decay,
                        max_grad_norm=cfg.max_grad_norm or 1.0, shard=shard)
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
