"""Bucketed data-parallel gradient reducer over RCCL (north-star N6 / N7).

Design (MI355X-first, not a DDP re-implementation):

* gradients already live in one flat arena (``optim.arena.ParamArena``) ordered
  in reverse registration order, so a *bucket* is just a contiguous slice of it:
  no flatten/unflatten copies, and the all-reduce payload is the gradient
  memory itself;
* bucket boundaries: a small first bucket (``first_bucket_mb``, default 4 MB) so
  the first RCCL ring starts while most of backward is still running, then
  ``bucket_mb`` buckets (default 25 MB: the last bucket's all-reduce is the
  exposed part, so it must stay small; bigger ones buy nothing) — an 8-GPU xGMI ring is
  per-link bound (~153 GB/s/link, 7 links), so few large messages that let RCCL
  spread channels over all links beat many small latency-bound ones;
* readiness: ``register_post_accumulate_grad_hook`` per parameter counts down a
  bucket; the last gradient of a bucket launches an async all-reduce, which
  ProcessGroupNCCL (RCCL) runs on its own HIP stream ordered after the
  producing kernels — comm overlaps the rest of backward;
* ``no_sync()`` for gradient accumulation (BASELINE.json:11): micro-steps skip
  communication; with ``accumulate_fp32`` the micro-step gradients are summed
  into an fp32 arena so bf16 accumulation error does not grow with grad_accum;
* the 1/world average is folded into the optimizer (``grad_scale``) instead of
  an extra pass over the buckets;
* ``shard=True`` (ZeRO-1, world > 1): each bucket is REDUCE-SCATTERED instead of
  all-reduced -- bucket boundaries are multiples of ``world * 64`` elements, rank r
  receives the reduced chunk r of every bucket into a local gradient shard, which is
  exactly the gradient its sharded optimizer (``optim.flat``, ``shard=(r, w, groups)``)
  updates.  After the step the updated chunks are ALL-GATHERED back per bucket on the
  comm stream (``gather_params``) in the order the next forward needs them (the last
  bucket holds the first layers), and a forward pre-hook per module waits for exactly
  the buckets holding that module's parameters: the gathers overlap the forward.
  Traffic per step equals one all-reduce (reduce-scatter + all-gather) instead of
  all-reduce + all-gather;
* ``comm="native"`` (default on GPU + RCCL) issues the bucket all-reduces
  through the C++ engine in ``csrc/runtime/comm.cpp`` (its own RCCL
  communicator and high-priority HIP stream, event-ordered after the producing
  kernels, one stream wait before the optimizer); ``comm="torch"`` uses
  ``torch.distributed.all_reduce(async_op=True)`` (gloo on CPU).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from . import dist as ddist
from ..optim.arena import ParamArena


@dataclass
class Bucket:
    index: int
    start: int
    end: int
    entry_ids: List[int]
    pending: int = 0
    handle: Optional[object] = None
    launched: bool = False
    payload: Optional[torch.Tensor] = None
    shard_off: int = 0           # ZeRO-1: this rank's chunk of the bucket in the local gradient shard
    grads_seen: set = field(default_factory=set)
    seq: int = 0                 # native engine: this bucket's all-reduce number (wait_upto)
    eager_done: bool = False     # set_eager callback already issued on the side stream


def _acc_grad(acc32: torch.Tensor, grad: torch.Tensor, first: bool, zero_grad: bool) -> None:
    """acc32 = grad (``first``: the accumulator's old contents are dead -- no zero fill per step) or
    acc32 += grad, then grad = 0 if ``zero_grad``: one native pass on the GPU (ddl_acc_grad, 16-byte
    vectors; it replaced an ATen mixed-dtype add per bucket and an fp32 zero fill of the whole
    accumulator per step, ~1 ms of BERT-large's step), ATen ops elsewhere."""
    if grad.is_cuda and grad.numel() % 8 == 0 and grad.dtype in (torch.bfloat16, torch.float32) and \
            acc32.data_ptr() % 16 == 0 and grad.data_ptr() % 16 == 0:
        from ..ops import _lib
        if _lib.use_native(grad):      # (False under --native off: the CPU-oracle mode)
            _lib.call("ddl_acc_grad", _lib.dcode(grad), acc32.data_ptr(), grad.data_ptr(), grad.numel(),
                      int(first), int(zero_grad))
            return
    if first:
        acc32.copy_(grad)
    else:
        acc32.add_(grad)
    if zero_grad:
        grad.zero_()


class ReplicaDivergence(RuntimeError):
    """Data-parallel replicas no longer hold identical parameters (see ``check_replicas``)."""


class DataParallel(nn.Module):
    """Wrap ``module`` for data-parallel training.

    ``arena`` may be supplied (shared with a flat optimizer); otherwise one is
    created.  After ``loss.backward()`` call :meth:`finish` (or use the
    optimizer's ``step(reducer=...)``), which waits on every in-flight bucket.
    """

    def __init__(self, module: nn.Module, arena: Optional[ParamArena] = None,
                 bucket_mb: float = 25.0, first_bucket_mb: float = 4.0,
                 reduce_dtype: Optional[torch.dtype] = None, broadcast_buffers: bool = False,
                 accumulate_fp32: bool = False, process_group=None, broadcast_init: bool = True,
                 comm: str = "auto", backward_passes_per_step: int = 1, shard: bool = False,
                 split_tensors: bool = True):
        super().__init__()
        self.module = module
        self.arena = arena if arena is not None else ParamArena(list(module.named_parameters()))
        self.pg = process_group
        self.world = ddist.world_size()
        self.broadcast_buffers = broadcast_buffers
        self.reduce_dtype = reduce_dtype or self.arena.dtype
        self.accumulate_fp32 = accumulate_fp32
        self._sync = True
        # Horovod semantics: a parameter's gradient is communicated on its k-th arrival
        # (k backward passes accumulate locally in the arena first); see _make_hook
        self.passes = max(1, int(backward_passes_per_step))
        self._arrivals: dict = {}
        self._acc32: Optional[torch.Tensor] = None
        self._acc_active = False
        if broadcast_init and self.world > 1:
            ddist.broadcast_tensors([self.arena.flat] + [b for b in module.buffers()])
        self.native = None
        if not isinstance(comm, str):        # an engine object (all_reduce / wait), e.g. for tests
            self.native = comm
        elif comm == "native" or (comm == "auto" and self.world > 1):
            from .comm import CommError, NativeComm, native_available
            if native_available() and self.arena.flat.is_cuda:
                try:
                    self.native = NativeComm(process_group)
                except CommError as e:
                    if comm == "native":
                        raise
                    # every rank reaches the same outcome (same library, same RCCL), so
                    # falling back keeps the collective sequence identical across ranks
                    import warnings
                    warnings.warn(f"native RCCL engine unavailable ({e}); using torch.distributed")
            elif comm == "native":
                raise RuntimeError("comm='native' needs CUDA tensors, the native library and the nccl backend")
        self.comm = "native" if self.native is not None else "torch"
        from . import comm as _comm
        # SyncBatchNorm and the sharded optimizer's norm reductions ride the reducer's
        # communicator; a reducer without one clears whatever an earlier reducer left active
        _comm.set_active(self.native if (self.native is not None and hasattr(self.native, "world")) else None)
        self.shard = bool(shard) and self.world > 1
        self.split_tensors = bool(split_tensors)
        self._last_step: List[tuple] = []     # (bucket index, engine seq) of the last finished step
        if self.shard:
            unit = self.world * 64
            if self.arena.numel % unit:
                raise ValueError("DataParallel(shard=True): build the arena with pad_multiple = world * 64")
            self.buckets = self._build_shard_buckets(bucket_mb, first_bucket_mb, unit)
        else:
            self.buckets = self._build_buckets(bucket_mb, first_bucket_mb)
        self._entry_buckets: dict = {}
        for b in self.buckets:
            for ei in b.entry_ids:
                self._entry_buckets.setdefault(ei, []).append(b.index)
        self._gshard: Optional[torch.Tensor] = None
        self._gather_marks: dict = {}        # bucket index -> native seq / torch handle of its all-gather
        self._prehooks = []
        if self.shard:
            self._install_gather_waits()
        self._eager_cb: Optional[Callable[[torch.Tensor, int, int], None]] = None
        self._eager_stream = None
        self._eager_used = False
        self._hooks = []
        for ei, e in enumerate(self.arena.entries):
            hook = self._make_hook(ei)
            self._hooks.append(e.param.register_post_accumulate_grad_hook(hook))
            # native backward kernels accumulate straight into the arena view and call this
            e.param._ddl_main_grad = self.arena.grad[e.offset:e.offset + e.numel].view(e.shape)
            e.param._ddl_grad_ready = (lambda h=hook, prm=e.param: h(prm, native=True))
        self._reset()

    # ------------------------------------------------------------------
    def _build_buckets(self, bucket_mb: float, first_bucket_mb: float) -> List[Bucket]:
        """Whole tensors per bucket, in arena order; a single tensor larger than a bucket
        (BERT's 47 MB word embedding) is cut into bucket-sized pieces of its own
        (``split_tensors``): they all launch when its gradient lands, and the per-bucket
        optimizer starts on the first piece while the later ones are still on the wire.
        Piece boundaries sit on the flat optimizer's 8192-element row grid (relative to the
        tensor's start), so a range step updates whole rows."""
        esz = torch.empty((), dtype=self.reduce_dtype).element_size()
        buckets: List[Bucket] = []
        cap = int(first_bucket_mb * (1 << 20)) // esz
        full = max(1, int(bucket_mb * (1 << 20)) // esz)
        cur: List[int] = []
        start = 0
        ents = self.arena.entries
        for ei, e in enumerate(ents):
            nxt = ents[ei + 1].offset if ei + 1 < len(ents) else self.arena.numel
            if self.split_tensors and e.numel > full:
                if cur:                            # close the bucket in progress first
                    buckets.append(Bucket(len(buckets), start, e.offset, cur))
                    cur, start = [], e.offset
                piece = -(-full // 8192) * 8192
                a = start
                while a < nxt:
                    b = nxt if nxt - (a + piece) < piece // 2 else a + piece   # no tiny tail piece
                    buckets.append(Bucket(len(buckets), a, b, [ei]))
                    a = b
                start = nxt
                cap = full
                continue
            end = e.offset + e.numel
            cur.append(ei)
            if end - start >= cap:
                buckets.append(Bucket(len(buckets), start, nxt, cur))
                cur, start = [], nxt
                cap = full
        if cur:
            buckets.append(Bucket(len(buckets), start, self.arena.numel, cur))
        return buckets

    def _build_shard_buckets(self, bucket_mb: float, first_bucket_mb: float, unit: int) -> List[Bucket]:
        """ZeRO-1 buckets: boundaries rounded UP to a multiple of ``unit`` = world * 64 elements
        (past the first tensor end that fills the bucket), so every rank's chunk is whole and
        64-aligned; a tensor may straddle two buckets (both wait for it)."""
        esz = torch.empty((), dtype=self.reduce_dtype).element_size()
        bounds, start = [], 0
        cap = int(first_bucket_mb * (1 << 20)) // esz
        for e in self.arena.entries:
            end = e.offset + e.numel
            if end - start >= cap:
                b = min(self.arena.numel, -(-end // unit) * unit)
                if b > start:
                    bounds.append((start, b))
                    start = b
                cap = int(bucket_mb * (1 << 20)) // esz
        if start < self.arena.numel:
            bounds.append((start, self.arena.numel))
        buckets, off = [], 0
        for i, (a, b) in enumerate(bounds):
            ids = [ei for ei, e in enumerate(self.arena.entries) if e.offset < b and e.offset + e.numel > a]
            bk = Bucket(i, a, b, ids)
            bk.shard_off = off
            off += (b - a) // self.world
            buckets.append(bk)
        return buckets

    def shard_groups(self) -> List[tuple]:
        """(start, end) of every bucket: the ``groups`` a sharded optimizer takes."""
        return [(b.start, b.end) for b in self.buckets]

    def _install_gather_waits(self) -> None:
        """Forward pre-hook per module: wait for the all-gathers of the buckets holding the
        parameters its forward may read (stream waits, no host sync).

        A fused op reads the parameters of modules whose own forward never runs (a
        bottleneck block hands ``bn3`` / ``downsample.bn`` to ``conv_bn_add_bn``; ResNet's
        stem and ViT's patch embedding are read by the root's forward), so a module waits for
        its WHOLE subtree's buckets by default -- any parameter a forward can reach is in
        its subtree.  Routers (the wrapped root, ``nn.Sequential`` / ``nn.ModuleList`` and
        modules with ``_ddl_gather_router = True``) only dispatch to children whose own hooks
        wait: they wait for their direct parameters plus the subtrees of the children named
        in ``_ddl_direct_reads`` -- that keeps a model's all-gathers overlapped with its
        forward instead of all waited for before the first layer."""
        index = {id(e.param): ei for ei, e in enumerate(self.arena.entries)}

        def buckets_of(params):
            bks = set()
            for prm in params:
                ei = index.get(id(prm))
                if ei is not None:
                    bks.update(self._entry_buckets.get(ei, []))
            return bks

        for mod in self.module.modules():
            router = mod is self.module or isinstance(mod, (nn.Sequential, nn.ModuleList)) or \
                bool(getattr(mod, "_ddl_gather_router", False))
            if router:
                bks = buckets_of(mod.parameters(recurse=False))
                for name in getattr(mod, "_ddl_direct_reads", ()):
                    bks |= buckets_of(getattr(mod, name).parameters())
            else:
                bks = buckets_of(mod.parameters())
            if bks:
                need = sorted(bks)
                self._prehooks.append(mod.register_forward_pre_hook(
                    lambda _m, _a, need=need: self._wait_gathers(need)))

    def _wait_gathers(self, idx) -> None:
        for i in idx:
            mark = self._gather_marks.pop(i, None)
            if mark is None:
                continue
            if isinstance(mark, int):
                self.native.wait_upto(mark)
            else:
                mark.wait()

    def wait_params(self) -> None:
        """Make the current stream wait for every outstanding parameter all-gather
        (before reading parameters outside a forward: checkpoints, evaluation)."""
        self._wait_gathers(list(self._gather_marks))

    def gather_params(self, groups, ranges) -> None:
        """Sharded optimizer's ``gather_fn``: all-gather every bucket's updated chunks into
        the arena, asynchronously, last bucket (the first layers) first."""
        flat = self.arena.flat
        order = sorted(range(len(groups)), key=lambda i: -groups[i][0])
        for i in order:
            (a, b), (lo, hi, _) = groups[i], ranges[i]
            if self.native is not None:
                self._gather_marks[i] = self.native.all_gather(flat[lo:hi], flat[a:b])
            else:
                send = flat[lo:hi] if flat.is_cuda else flat[lo:hi].clone()
                self._gather_marks[i] = dist.all_gather_into_tensor(flat[a:b], send, group=self.pg, async_op=True)

    def _reset(self) -> None:
        for b in self.buckets:
            b.pending = len(b.entry_ids)
            b.handle = None
            b.launched = False
            b.payload = None
            b.grads_seen = set()
            b.seq = 0
            b.eager_done = False
        self._order: List[Bucket] = []       # buckets in all-reduce launch order
        self._arrivals = {}
        self._native_seen: set = set()

    def _make_hook(self, ei: int):
        # Ordering rule for native backward ops (grad_sink / grad_ready): an op calls
        # grad_ready(param) only AFTER the last kernel of this backward that reads the
        # parameter (dgrad before wgrad; BN / LN read gamma before reporting it).  With the
        # eager optimizer on, the bucket's update runs on a side stream from that point
        # and rewrites the weight.
        def hook(_p, native: bool = False):
            # a native backward reports through grad_ready (native=True) and autograd's
            # post-accumulate hook then fires for the same parameter (its returned gradient
            # is None): the second, autograd, report is the expected echo
            if not self._sync:
                return
            if native:
                if ei in self._native_seen and self._eager_cb is not None and \
                        any(self.buckets[bi].launched for bi in self._entry_buckets[ei]):
                    # two native uses of one weight in one step: the side stream may already be
                    # rewriting it while the second use's backward still reads it -- refuse
                    raise RuntimeError(
                        f"parameter {self.arena.entries[ei].name} reported its gradient twice in one step "
                        "with the eager optimizer on; turn eager_optimizer off for this model")
                self._native_seen.add(ei)
            elif ei in self._native_seen:
                return
            if self.passes > 1:
                n = self._arrivals.get(ei, 0) + 1
                self._arrivals[ei] = n
                if n < self.passes:          # accumulate locally; communicate on pass k
                    return
            for bi in self._entry_buckets[ei]:
                b = self.buckets[bi]
                if ei in b.grads_seen:   # parameter used twice in one graph: count once
                    continue
                b.grads_seen.add(ei)
                b.pending -= 1
                if b.pending == 0:
                    self._launch(b)
        return hook

    def _payload(self, b: Bucket) -> torch.Tensor:
        g = self.arena.grad[b.start:b.end]
        if self._acc_active:
            acc = self._acc32[b.start:b.end]
            _acc_grad(acc, g, first=False, zero_grad=False)
            return acc
        if self.reduce_dtype != g.dtype:
            return g.to(self.reduce_dtype)
        return g

    def _launch(self, b: Bucket) -> None:
        if b.launched:
            return
        b.launched = True
        self._order.append(b)
        b.payload = self._payload(b)
        if self.shard:
            self._launch_scatter(b)
            return
        if self.native is not None or self.world > 1:
            if self.native is not None:
                # payload is the arena slice / fp32 accumulator / a converted copy held
                # in b.payload until finish() -- alive until the comm stream is drained
                seq = self.native.all_reduce(b.payload)
                b.seq = seq if isinstance(seq, int) else 0
            else:
                b.handle = dist.all_reduce(b.payload, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
        if self._eager_cb is not None and self._eager_ok():
            self._run_eager(b)

    def _launch_scatter(self, b: Bucket) -> None:
        """ZeRO-1: reduce-scatter the bucket; chunk ``rank`` lands in the local gradient shard."""
        n = (b.end - b.start) // self.world
        if self._gshard is None or self._gshard.dtype != b.payload.dtype:
            self._gshard = torch.empty(self.arena.numel // self.world, dtype=b.payload.dtype, device=self.arena.device)
        recv = self._gshard[b.shard_off:b.shard_off + n]
        if self.native is not None:
            b.seq = self.native.reduce_scatter(b.payload, recv)
        else:
            b.handle = dist.reduce_scatter_tensor(recv, b.payload, group=self.pg, async_op=True)

    # ------------------------------------------------------------------ eager per-bucket callbacks
    def _eager_ok(self) -> bool:
        return (not self.shard and self.arena.grad.is_cuda and self.reduce_dtype == self.arena.dtype and not self._acc_active
                and (self.native is None or hasattr(self.native, "wait_upto")))

    def set_eager(self, cb: Optional[Callable[[torch.Tensor, int, int], None]]) -> None:
        """Run ``cb(grad, lo, hi)`` for each bucket DURING backward, the moment the bucket's
        gradients exist (and, with several ranks, its all-reduce is done), on a side stream:
        the flat optimizer's HBM-bound update of the late layers then runs under the early
        layers' backward GEMMs instead of after the whole backward.  :meth:`finish` joins the
        side stream back into the compute stream.  ``None`` turns it off."""
        self._eager_cb = cb
        if cb is not None and self._eager_stream is None and self.arena.grad.is_cuda:
            self._eager_stream = torch.cuda.Stream(device=self.arena.grad.device)

    def _run_eager(self, b: Bucket) -> None:
        compute = torch.cuda.current_stream(self.arena.grad.device)
        side = self._eager_stream
        side.wait_stream(compute)               # every kernel that produced this bucket's gradients
        with torch.cuda.stream(side):
            if b.handle is not None:
                b.handle.wait()                 # the side stream waits for this bucket's ring
            elif self.native is not None and b.seq > 0:
                self.native.wait_upto(b.seq)
            self._eager_cb(self.arena.grad, b.start, b.end)
        b.eager_done = True
        self._eager_used = True

    # ------------------------------------------------------------------
    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        """Skip gradient communication inside (micro-steps of grad accumulation)."""
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev
            if self.accumulate_fp32:
                # drain this micro-step's bf16 grads into the fp32 accumulator
                if self._acc32 is None:
                    self._acc32 = torch.empty(self.arena.numel, dtype=torch.float32, device=self.arena.device)
                _acc_grad(self._acc32, self.arena.grad, first=not self._acc_active, zero_grad=True)
                self._acc_active = True

    def replica_fingerprint(self, chunk: int = 1 << 22) -> torch.Tensor:
        """fp64 [sum, position-weighted sum] of this rank's parameter arena (2 numbers per
        check; weighted so a permutation or a swapped bucket does not cancel out).

        Walked in ``chunk``-element pieces (fp32 partial sums per piece, accumulated in
        fp64) with a period-4093 weight pattern built once, so a check costs a few MB of
        scratch instead of an fp64 copy of the whole arena."""
        flat = self.arena.flat.detach()
        n = flat.numel()
        period = 4093
        chunk = max(period, chunk - chunk % period)      # every piece starts on a weight period
        base = torch.arange(1, chunk + 1, device=flat.device, dtype=torch.float32).remainder_(float(period)).add_(1.0)
        s = torch.zeros((), dtype=torch.float64, device=flat.device)
        ws = torch.zeros((), dtype=torch.float64, device=flat.device)
        for lo in range(0, n, chunk):
            x = flat[lo:lo + chunk].float()
            s += x.sum(dtype=torch.float64)
            ws += (x * base[:x.numel()]).sum(dtype=torch.float64)
        return torch.stack([s, ws])

    def check_replicas(self, rtol: float = 0.0) -> None:
        """Debug / race check: data-parallel replicas must hold IDENTICAL parameters
        after every optimizer step (same all-reduced gradient, same update).  A missing stream
        dependency -- an optimizer reading a bucket before its all-reduce landed, an eager update
        racing a backward read -- shows up as replicas drifting apart.  All ranks call this at
        the same step; every rank raises ``ReplicaDivergence`` when fingerprints differ."""
        if self.world == 1:
            return
        self.wait_params()
        fp = self.replica_fingerprint()
        lo, hi = fp.clone(), fp.clone()
        if not fp.is_cuda or dist.get_backend(self.pg) == "gloo":
            lo, hi = lo.cpu(), hi.cpu()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.pg)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.pg)
        spread = (hi - lo).abs().cpu()
        scale = torch.maximum(hi.abs(), lo.abs()).cpu()
        if bool((spread > rtol * scale).any()):
            raise ReplicaDivergence(f"rank {ddist.rank()}: parameter replicas differ across ranks "
                                    f"(fingerprint min {lo.tolist()} max {hi.tolist()})")

    def finish(self, on_ready: Optional[Callable[[torch.Tensor, int, int], None]] = None) -> torch.Tensor:
        """Wait for all buckets; return the flat reduced gradient (SUM over ranks).

        The caller scales by ``1/world`` (optimizers take ``grad_scale``).

        ``on_ready(grad, lo, hi)``: called per bucket in all-reduce order once the compute
        stream has been made to wait for THAT bucket only, with the arena index range it
        covers -- a range-stepping optimizer updates the early buckets while the last
        all-reduces (the embedding's, in BERT) are still on the wire.
        """
        self.wait_params()           # a step without a forward in between still sees gathered params
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        self._last_step = [(b.index, b.seq) for b in self._order]
        if self.shard:
            for b in self.buckets:
                if b.handle is not None:
                    b.handle.wait()
            if self.native is not None:
                self.native.wait()
            out = self._gshard
            self._reset()
            return out
        if self._eager_used:
            # the callbacks ran during backward on the side stream: the compute stream (next
            # forward, zero_grad) waits for them; the rings were waited for on the side stream
            torch.cuda.current_stream(self.arena.grad.device).wait_stream(self._eager_stream)
            on_ready = None
            self._eager_used = False
        elif self._eager_cb is not None and on_ready is None:
            on_ready = self._eager_cb           # requested but not possible this step: per bucket, now
        streamed = on_ready is not None and self.reduce_dtype == self.arena.dtype
        out_early = self._acc32 if self._acc_active else self.arena.grad
        if streamed:
            can_seq = self.native is not None and hasattr(self.native, "wait_upto") and \
                all(b.seq > 0 for b in self._order if b.end > b.start)
            if self.native is not None and not can_seq:
                self.native.wait()          # engine without per-collective marks: one wait
            for b in self._order:
                if b.handle is not None:
                    b.handle.wait()
                elif self.native is not None and can_seq:
                    self.native.wait_upto(b.seq)
                on_ready(out_early, b.start, b.end)
        else:
            for b in self.buckets:
                if b.handle is not None:
                    b.handle.wait()
        if self.native is not None:
            self.native.wait()
        if self._acc_active:
            out = self._acc32
        elif self.reduce_dtype != self.arena.dtype:
            out = torch.empty(self.arena.numel, dtype=self.reduce_dtype, device=self.arena.device)
            for b in self.buckets:
                out[b.start:b.end].copy_(b.payload)
        else:
            out = self.arena.grad
        self._reset()
        if self.broadcast_buffers and self.world > 1:
            ddist.broadcast_tensors(list(self.module.buffers()))
        return out

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.arena.zero_grad()
        # (the fp32 accumulator is not cleared: the next step's first drain overwrites it)
        self._acc_active = False

    def bucket_timings(self) -> List[dict]:
        """Per bucket of the last finished step, in launch order: size, device time of its
        collective on the comm stream (start -> done events of the native engine) and the bus
        bandwidth that implies (x 2(n-1)/n for an all-reduce, (n-1)/n for a reduce-scatter).
        Empty without the native engine (torch / gloo path) or before the first step.  Reads
        events only: call it after the step's work has been synchronised."""
        eng = self.native
        if eng is None or not hasattr(eng, "collective_ms"):
            return []
        esz = torch.empty((), dtype=self.reduce_dtype).element_size()
        n = max(1, self.world)
        factor = (n - 1) / n if self.shard else 2 * (n - 1) / n
        out = []
        for bi, seq in self._last_step:
            b = self.buckets[bi]
            mb = (b.end - b.start) * esz / (1 << 20)
            ms = eng.collective_ms(seq) if seq > 0 else -1.0
            bus = (b.end - b.start) * esz * factor / (ms * 1e-3) / 1e9 if ms > 0 else None
            out.append({"bucket": bi, "mb": round(mb, 2), "ms": round(ms, 4) if ms >= 0 else None,
                        "busbw_gbs": round(bus, 1) if bus else None})
        return out

    def bucket_sizes_mb(self) -> List[float]:
        esz = torch.empty((), dtype=self.reduce_dtype).element_size()
        return [(b.end - b.start) * esz / (1 << 20) for b in self.buckets]

    def close(self, abort: bool = False) -> None:
        """Release the reducer: remove its hooks and destroy its native communicator (which
        also clears it as the process's active engine).  ``abort``: the failure path
        (``ncclCommAbort``, no waiting on peers)."""
        for h in self._hooks + self._prehooks:
            h.remove()
        self._hooks, self._prehooks = [], []
        if self.native is not None and hasattr(self.native, "close"):
            self.native.close(abort=abort)
        from . import comm as _comm
        if _comm.active() is self.native:
            _comm.set_active(None)
        self.native = None

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, *a, **k):
        return self.module.load_state_dict(*a, **k)
