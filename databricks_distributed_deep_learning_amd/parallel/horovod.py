"""HorovodRunner-compatible shim + a tiny ``hvd``-style facade (north-star N2).

``HorovodRunner(np=8).run(main, **kwargs)`` mirrors the public
``sparkdl.HorovodRunner`` surface; negative ``np`` (Databricks' "run locally on
the driver with |np| processes") is treated the same as positive on one node.
The facade (``init/rank/size/local_rank/allreduce/allgather/broadcast/
broadcast_parameters/broadcast_optimizer_state/DistributedOptimizer``) is backed
by ``torch.distributed`` over RCCL and by :class:`..parallel.ddp.DataParallel`'s
bucketed reducer, so Horovod-style training scripts run unchanged in structure.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Iterable, Optional

import torch
import torch.distributed as dist

from . import dist as ddist
from .launcher import Distributor

Average = "average"
Sum = "sum"
Adasum = "adasum"  # scale-invariant pairwise combination (``adasum_combine``), not an average


class HorovodRunner:
    def __init__(self, np: int = -1, driver_log_verbosity: str = "log_callback_only", use_gpu: Optional[bool] = None):
        self.num_processes = abs(int(np)) or 1
        self.driver_log_verbosity = driver_log_verbosity
        self.use_gpu = use_gpu

    def run(self, main: Callable, **kwargs) -> Any:
        return Distributor(self.num_processes, local_mode=True, use_gpu=self.use_gpu).run(main, **kwargs)


# ---------------------------------------------------------------- facade
def init(backend: str = "auto") -> None:
    ddist.init(backend=backend)


def rank() -> int:
    return ddist.rank()


def size() -> int:
    return ddist.world_size()


def local_rank() -> int:
    return ddist.local_rank()


def local_size() -> int:
    import os
    return int(os.environ.get("LOCAL_WORLD_SIZE", size()))


def _prep(t: torch.Tensor):
    if ddist.is_initialized() and dist.get_backend() == "nccl" and not t.is_cuda:
        return t.cuda(), True
    return t, False


def adasum_combine(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Horovod's Adasum of two gradients: ``(1 - a.b / 2|a|^2) a + (1 - a.b / 2|b|^2) b``.

    Orthogonal gradients add, identical ones average, and the result does not change
    when either input is scaled -- the property that lets Adasum keep the learning rate
    of a single worker as the worker count grows.  Dot products in fp64."""
    a64, b64 = a.double(), b.double()
    dot = (a64 * b64).sum()
    na, nb = (a64 * a64).sum(), (b64 * b64).sum()
    ca = torch.where(na > 0, 1.0 - dot / (2.0 * na), torch.ones_like(na))
    cb = torch.where(nb > 0, 1.0 - dot / (2.0 * nb), torch.ones_like(nb))
    return (ca * a64 + cb * b64).to(a.dtype)


def adasum_tree(parts) -> torch.Tensor:
    """Adasum over ranks in Horovod's recursive-doubling order: (0,1), (2,3), ... then
    the pairs of pairs; an odd one out is carried up a level unchanged."""
    parts = list(parts)
    while len(parts) > 1:
        parts = [adasum_combine(parts[i], parts[i + 1]) if i + 1 < len(parts) else parts[i]
                 for i in range(0, len(parts), 2)]
    return parts[0]


def _combine_segments(lower: torch.Tensor, upper: torch.Tensor, segments) -> torch.Tensor:
    """adasum_combine(lower, upper) applied to each (offset, numel) segment independently."""
    out = torch.empty_like(lower)
    for off, n in segments:
        out[off:off + n] = adasum_combine(lower[off:off + n], upper[off:off + n])
    return out


def _exchange(send: torch.Tensor, to, recv: torch.Tensor, frm: int) -> None:
    """Send ``send`` to every rank in ``to`` and receive ``recv`` from ``frm`` (one batch: the
    RCCL backend needs the pair's send and receive grouped, or both sends block)."""
    ops = [dist.P2POp(dist.isend, send, q) for q in to] + [dist.P2POp(dist.irecv, recv, frm)]
    for req in dist.batch_isend_irecv(ops):
        req.wait()


def adasum_allreduce(tensor: torch.Tensor, segments: Optional[Iterable] = None) -> torch.Tensor:
    """Adasum of ``tensor`` over all ranks, identical on every rank, by recursive doubling:
    at level l (stride s = 2^l) rank blocks of s ranks -- each block holding its Adasum so far --
    pair with the neighbouring block (b, b ^ 1); every rank swaps its vector with one rank of the
    partner block and both compute ``adasum_combine(lower block, upper block)`` (Horovod's
    order: (0,1), (2,3), ... then pairs of pairs, = ``adasum_tree``); a block with no partner
    is carried up unchanged.  Memory is O(numel) per rank (one receive buffer), not
    world x numel.  ``segments`` = (offset, numel) ranges combined independently (Horovod
    applies Adasum per tensor); default: the whole tensor."""
    n, r = size(), rank()
    cur = tensor.reshape(-1).contiguous().clone()
    segs = list(segments or [(0, cur.numel())])
    if n == 1:
        return cur.view_as(tensor)
    buf = torch.empty_like(cur)
    s = 1
    while s < n:
        b, nblocks = r // s, -(-n // s)
        pb = b ^ 1
        if pb < nblocks:
            first, bsize = b * s, min(s, n - b * s)
            pfirst, psize = pb * s, min(s, n - pb * s)
            frm = pfirst + min(r - first, psize - 1)          # my source in the partner block
            to = [pfirst + j for j in range(psize) if first + min(j, bsize - 1) == r]
            _exchange(cur, to, buf, frm)
            lower, upper = (cur, buf) if b < pb else (buf, cur)
            cur = _combine_segments(lower, upper, segs)
        s *= 2
    return cur.view_as(tensor)


def allreduce(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
              op: str = Average) -> torch.Tensor:
    if average is not None:
        op = Average if average else Sum
    if op not in (Average, Sum, Adasum):
        raise ValueError(f"unknown reduction op {op!r}")
    out = tensor.detach().clone()
    if size() == 1:
        return out
    t, moved = _prep(out)
    if op == Adasum:
        t = adasum_allreduce(t)
    else:
        dist.all_reduce(t)
        if op == Average:
            t.div_(size())
    return t.to(tensor.device) if moved else t


def allreduce_(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
               op: str = Average) -> torch.Tensor:
    tensor.copy_(allreduce(tensor, average=average, op=op))
    return tensor


def allgather(tensor: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    """Concatenate along dim 0 (Horovod semantics; equal first dims)."""
    if size() == 1:
        return tensor.detach().clone()
    t, moved = _prep(tensor.detach().contiguous())
    outs = [torch.empty_like(t) for _ in range(size())]
    dist.all_gather(outs, t)
    r = torch.cat(outs, 0)
    return r.to(tensor.device) if moved else r


def broadcast(tensor: torch.Tensor, root_rank: int = 0, name: Optional[str] = None) -> torch.Tensor:
    out = tensor.detach().clone()
    if size() == 1:
        return out
    t, moved = _prep(out)
    dist.broadcast(t, src=root_rank)
    return t.to(tensor.device) if moved else t


def broadcast_(tensor: torch.Tensor, root_rank: int = 0, name: Optional[str] = None) -> torch.Tensor:
    tensor.copy_(broadcast(tensor, root_rank))
    return tensor


def broadcast_parameters(params, root_rank: int = 0) -> None:
    if isinstance(params, dict):
        tensors = list(params.values())
    else:
        tensors = [p for _, p in params] if params and isinstance(next(iter(params)), tuple) else list(params)
    with torch.no_grad():
        ddist.broadcast_tensors([t.data if hasattr(t, "data") else t for t in tensors], src=root_rank)


def broadcast_object(obj: Any, root_rank: int = 0) -> Any:
    return ddist.broadcast_object(obj, src=root_rank)


def broadcast_optimizer_state(optimizer, root_rank: int = 0) -> None:
    sd = optimizer.state_dict()
    sd = ddist.broadcast_object(sd, src=root_rank)
    optimizer.load_state_dict(sd)


class _DistributedOptimizer:
    """Wraps a torch optimizer: averages gradients across ranks before ``step``.

    Communication is bucketed and overlapped with backward through the same
    hook-driven reducer as :class:`DataParallel` (grads are views into one flat
    arena, all-reduced slice by slice as they become ready).

    ``op=Adasum`` follows Horovod's Adasum optimizer: every rank takes a LOCAL optimizer step
    on its own gradient, and the parameter deltas (not the raw gradients) are combined with
    Adasum per tensor (:func:`adasum_allreduce`, recursive doubling); the parameters become
    ``p_before + adasum(delta)``.  For plain SGD this equals Adasum of the gradients (times
    -lr); with momentum / Adam the two differ, and this is the one Horovod computes.
    (Horovod itself is not importable here: the parity is with its documented algorithm.)
    """

    def __init__(self, optimizer: torch.optim.Optimizer, named_parameters: Optional[Iterable] = None,
                 backward_passes_per_step: int = 1, op: str = Average, bucket_mb: float = 64.0):
        from .ddp import DataParallel
        from ..optim.arena import ParamArena
        self.optimizer = optimizer
        if named_parameters is None:
            named_parameters = [(f"p{i}", p) for g in optimizer.param_groups for i, p in enumerate(g["params"])]
        self.arena = ParamArena(list(named_parameters))

        class _Holder(torch.nn.Module):
            pass
        if op not in (Average, Sum, Adasum):
            raise ValueError(f"unknown reduction op {op!r}")
        self.op = op
        self.backward_passes_per_step = backward_passes_per_step
        if op == Adasum:
            # gradients stay local (accumulated in the arena); step() combines the deltas
            self.arena.rebind_grads()
            self._reducer = None
            return
        # backward_passes_per_step = k: each gradient is all-reduced on its k-th arrival
        # (the reducer counts per parameter, as Horovod does); passes 1..k-1 accumulate
        # locally into the arena and launch nothing
        self._reducer = DataParallel(_Holder(), arena=self.arena, bucket_mb=bucket_mb, broadcast_init=False,
                                     backward_passes_per_step=backward_passes_per_step)

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    def zero_grad(self, set_to_none: bool = False) -> None:
        if self._reducer is None:
            self.arena.zero_grad()
        else:
            self._reducer.zero_grad()

    def synchronize(self) -> None:
        if self._reducer is None:       # Adasum: nothing to reduce before the local step
            self.arena.rebind_grads()   # gradients a set_to_none zero_grad detached from the arena
            return
        self._reducer.finish()
        if self.op == Average and size() > 1:
            self.arena.grad.mul_(1.0 / size())

    def step(self, closure=None):
        self.synchronize()
        if self._reducer is not None or size() == 1:
            return self.optimizer.step(closure)
        # Adasum: local step, then p = p_before + Adasum over ranks of (p_after - p_before)
        before = self.arena.flat.detach().clone()
        loss = self.optimizer.step(closure)
        with torch.no_grad():
            delta = self.arena.flat - before
            d, moved = _prep(delta)
            segs = [(e.offset, e.numel) for e in self.arena.entries]
            out = adasum_allreduce(d, segs)
            self.arena.flat.copy_(before + (out.to(before.device) if moved else out))
        self.arena.bump()
        return loss

    def state_dict(self):
        return self.optimizer.state_dict()

    def load_state_dict(self, sd):
        return self.optimizer.load_state_dict(sd)


def DistributedOptimizer(optimizer, named_parameters=None, backward_passes_per_step: int = 1,
                         op: str = Average, **kw) -> _DistributedOptimizer:
    return _DistributedOptimizer(optimizer, named_parameters, backward_passes_per_step, op, **kw)
