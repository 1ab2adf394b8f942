"""Native RCCL comm engine binding (csrc/runtime/comm.cpp; SURVEY T-L0c / N6).

``NativeComm`` owns an RCCL communicator and a high-priority HIP stream of its
own.  The gradient reducer (``parallel/ddp.py``) calls :meth:`all_reduce` on
contiguous slices of the flat gradient arena the moment a bucket's last
gradient is produced; the engine orders the collective after the producing
kernels with an event (no host sync) and :meth:`wait` makes the compute stream
wait for all issued collectives before the optimizer step.

The unique id is created by rank 0 and distributed over the existing
``torch.distributed`` group (a 128-byte object), so the engine works under the
same launchers (``Distributor``, ``torchrun``) as everything else.  RCCL itself
is the library PyTorch loaded (``torch/lib/librccl.so``), resolved with dlopen.

Failure detection: a :class:`CommWatchdog` thread polls the engine's RCCL
asynchronous error state and the age of the oldest unfinished collective; on a peer failure
or a collective older than ``DDL_COMM_TIMEOUT_S`` (default 600 s, 0 = off) it aborts the
communicator (``ncclCommAbort``: RCCL kernels blocked on a dead peer return, the streams
drain) and every later engine call raises :class:`CommError` with the reason -- instead of
the rank hanging until the process-group timeout.

Bucket policy: :func:`probe_allreduce` times all-reduces of 1 / 4 / 16 / 64 MB
on the engine (bus bandwidth per size), :func:`fit_latency_bandwidth` fits
``t(S) = alpha + S / beta`` and :func:`auto_buckets` turns that into ``first_bucket_mb`` /
``bucket_mb`` for ``--bucket-mb auto``.
"""
from __future__ import annotations

import ctypes
import glob
import os
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops import _lib

I, L, P = ctypes.c_int, ctypes.c_long, ctypes.c_void_p
_SIGS = {
    "ddl_comm_unique_id": ([ctypes.c_char_p, ctypes.c_char_p], I),
    "ddl_comm_create": ([ctypes.c_char_p, ctypes.c_char_p, I, I, I], P),
    "ddl_comm_allreduce": ([P, P, L, I, I, P], I),
    "ddl_comm_allreduce_many": ([P, ctypes.POINTER(P), ctypes.POINTER(L), I, I, I, P], I),
    "ddl_comm_broadcast": ([P, P, L, I, I, P], I),
    "ddl_comm_reduce_scatter": ([P, P, P, L, I, I, P], I),
    "ddl_comm_all_gather": ([P, P, P, L, I, P], I),
    "ddl_comm_wait": ([P, P], I),
    "ddl_comm_wait_upto": ([P, L, P], I),
    "ddl_comm_synchronize": ([P], I),
    "ddl_comm_stats": ([P, I], L),
    "ddl_comm_destroy": ([P, I], None),
    "ddl_comm_last_error": ([], ctypes.c_char_p),
    "ddl_comm_async_error": ([P], I),
    "ddl_comm_oldest_pending_ms": ([P], ctypes.c_double),
    "ddl_comm_collective_ms": ([P, L], ctypes.c_double),
    "ddl_comm_abort": ([P], I),
    "ddl_comm_inject_error": ([P, I], I),
    "ddl_comm_test_stall": ([P, I], I),
    "ddl_comm_nonblocking": ([P], I),
}
_DTYPES = {torch.bfloat16: 0, torch.float32: 1, torch.float16: 2, torch.int64: 3, torch.int32: 4}


class CommError(RuntimeError):
    pass


# The engine the data-parallel reducer of this process drives (set by DataParallel).
# Other in-backward collectives (SyncBatchNorm statistics) go through the SAME
# communicator and stream, so only one RCCL communicator carries traffic while
# gradient buckets are in flight: two communicators whose kernels interleave in
# different orders on different ranks can deadlock once the CUs are full.
_ACTIVE: Optional["NativeComm"] = None


def set_active(engine: Optional["NativeComm"]) -> None:
    global _ACTIVE
    _ACTIVE = engine


def active() -> Optional["NativeComm"]:
    return _ACTIVE


def _fn(name):
    lib = _lib.get()
    f = getattr(lib, name)
    if not getattr(f, "_ddl_typed", False):
        args, res = _SIGS[name]
        f.argtypes = args
        f.restype = res
        f._ddl_typed = True
    return f


def rccl_path() -> str:
    """The librccl PyTorch loaded (fallback: the ROCm install)."""
    cands = glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so*"))
    cands += glob.glob("/opt/rocm/lib/librccl.so*")
    if not cands:
        raise CommError("librccl.so not found")
    return cands[0]


def _err() -> str:
    return (_fn("ddl_comm_last_error")() or b"").decode(errors="replace")


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def native_available() -> bool:
    return torch.cuda.is_available() and _lib.available() and dist.is_initialized() and \
        dist.get_backend() == "nccl"


class CommWatchdog:
    """Background thread: ``engine.poll()`` every ``interval`` seconds; the first error it
    returns aborts the engine (``engine.fail(reason)``) and stops the thread.

    ``engine`` needs ``poll() -> Optional[str]`` and ``fail(str)`` (NativeComm has both; the
    CPU tests drive a fake)."""

    def __init__(self, engine, interval: float = 1.0):
        self.engine = engine
        self.interval = max(0.01, float(interval))
        self._stop = threading.Event()
        self.reason: Optional[str] = None
        self._t = threading.Thread(target=self._loop, name="ddl-comm-watchdog", daemon=True)
        self._t.start()

    def _loop(self) -> None:
        while not self._stop.wait(self.interval):
            try:
                reason = self.engine.poll()
            except Exception as e:  # noqa: BLE001 - a failing poll is itself the failure
                reason = f"watchdog poll failed: {e}"
            if reason:
                self.reason = reason
                self.engine.fail(reason)
                return

    def stop(self) -> None:
        self._stop.set()
        if self._t is not threading.current_thread():
            self._t.join(timeout=5.0)


class NativeComm:
    """RCCL communicator over all ranks of ``group`` (default: the world).

    ``timeout_s``: a collective unfinished for longer is declared hung and the communicator
    aborted by the watchdog (env ``DDL_COMM_TIMEOUT_S``, default 600; 0 = no watchdog)."""

    def __init__(self, group=None, device: Optional[torch.device] = None, timeout_s: Optional[float] = None,
                 poll_s: Optional[float] = None):
        if not torch.cuda.is_available():
            raise CommError("NativeComm needs a GPU")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        path = rccl_path().encode()
        uid = ctypes.create_string_buffer(128)
        payload = None
        if self.rank == 0:
            rc = _fn("ddl_comm_unique_id")(path, uid)
            payload = uid.raw if rc == 0 else f"ddl_comm_unique_id failed: {_err()}"
        # rank 0 always broadcasts (the id or its error) so no rank is left waiting
        obj = [payload]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        if isinstance(obj[0], str):
            raise CommError(obj[0])
        self._h = _fn("ddl_comm_create")(path, obj[0], self.world, self.rank, self.device.index)
        ok = torch.tensor([1 if self._h else 0], device=self.device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if not self._h or int(ok.item()) == 0:
            raise CommError(f"ddl_comm_create failed on some rank: {_err() if not self._h else 'peer'}")
        self.failed: Optional[str] = None
        self.timeout_s = float(os.environ.get("DDL_COMM_TIMEOUT_S", "600") if timeout_s is None else timeout_s)
        interval = float(os.environ.get("DDL_COMM_POLL_S", "1.0") if poll_s is None else poll_s)
        self.watchdog = CommWatchdog(self, interval) if self.timeout_s > 0 else None

    # ------------------------------------------------------------------
    def _check(self, rc: int, what: str) -> None:
        if self.failed:
            raise CommError(f"{what}: communicator aborted ({self.failed})")
        if rc != 0:
            raise CommError(f"{what} failed ({rc}): {_err()}")

    def poll(self) -> Optional[str]:
        """The watchdog's check: an RCCL asynchronous error, or a collective on the comm
        stream for longer than ``timeout_s``; None while healthy."""
        h = getattr(self, "_h", None)
        if not h or self.failed:
            return None
        rc = int(_fn("ddl_comm_async_error")(h))
        if rc == -4:
            return None                       # aborted / closed meanwhile
        if rc != 0:
            return f"RCCL asynchronous error {rc} on rank {self.rank} (a peer failed or a connection broke)"
        age = float(_fn("ddl_comm_oldest_pending_ms")(h))
        if self.timeout_s > 0 and age > 1e3 * self.timeout_s:
            return f"collective on rank {self.rank} unfinished after {age / 1e3:.1f} s (timeout {self.timeout_s:g} s)"
        return None

    def fail(self, reason: str) -> None:
        """Abort the communicator from any thread; later calls raise CommError(reason)."""
        self.failed = reason
        h = getattr(self, "_h", None)
        if h:
            _fn("ddl_comm_abort")(h)

    def inject_error(self, code: int) -> None:
        """Test hook: make RCCL's asynchronous error state read ``code`` (the watchdog's input)."""
        _fn("ddl_comm_inject_error")(self._h, int(code))

    def stall_next_enqueue(self, ms: int) -> None:
        """Test hook: the next collective call blocks ``ms`` inside the engine, as an RCCL enqueue
        stuck in connection setup to a dead peer does (the watchdog must still see and abort it)."""
        _fn("ddl_comm_test_stall")(self._h, int(ms))

    @property
    def nonblocking(self) -> bool:
        """True when the communicator was created non-blocking (RCCL calls never block inside
        RCCL; an abort waits for no thread stuck there -- ``csrc/runtime/comm.cpp`` header)."""
        h = getattr(self, "_h", None)
        return bool(h) and bool(_fn("ddl_comm_nonblocking")(h))

    def collective_ms(self, seq: int) -> float:
        """Device time of finished collective ``seq`` (its start / done events), -1 if unknown."""
        h = getattr(self, "_h", None)
        if not h or seq <= 0:
            return -1.0
        return float(_fn("ddl_comm_collective_ms")(h, int(seq)))

    def all_reduce(self, t: torch.Tensor, average: bool = False) -> int:
        """In-place all-reduce of a contiguous GPU tensor on the comm stream (async).
        Returns its sequence number for :meth:`wait_upto` (0: nothing was issued).

        The number is read back from the engine (``ddl_comm_stats``), never mirrored in
        Python: a call that fails after the engine counted it must not leave a stale
        count behind that would make a later ``wait_upto`` wait on an older collective."""
        assert t.is_cuda and t.is_contiguous()
        self._check(_fn("ddl_comm_allreduce")(self._h, t.data_ptr(), t.numel(), _DTYPES[t.dtype], int(average),
                                              _stream()), "all_reduce")
        return self.collectives_launched if t.numel() > 0 else 0

    def all_reduce_many(self, ts: Sequence[torch.Tensor], average: bool = False) -> int:
        if not ts:
            return 0
        dt = ts[0].dtype
        assert all(t.dtype == dt and t.is_contiguous() for t in ts)
        bufs = (P * len(ts))(*[t.data_ptr() for t in ts])
        counts = (L * len(ts))(*[t.numel() for t in ts])
        self._check(_fn("ddl_comm_allreduce_many")(self._h, bufs, counts, len(ts), _DTYPES[dt], int(average),
                                                   _stream()), "all_reduce_many")
        return self.collectives_launched

    def wait_upto(self, seq: int) -> None:
        """Current (compute) stream waits for all-reduce number ``seq`` and every earlier
        collective: the optimizer can start on a bucket while later ones are in flight."""
        if seq > 0:
            self._check(_fn("ddl_comm_wait_upto")(self._h, int(seq), _stream()), "wait_upto")

    def broadcast(self, t: torch.Tensor, root: int = 0) -> None:
        self._check(_fn("ddl_comm_broadcast")(self._h, t.data_ptr(), t.numel(), _DTYPES[t.dtype], root, _stream()),
                    "broadcast")

    def reduce_scatter(self, send: torch.Tensor, recv: torch.Tensor, average: bool = False) -> int:
        """``recv`` = this rank's 1/world chunk of the sum of ``send`` over ranks (async on
        the comm stream); returns its sequence number for :meth:`wait_upto`."""
        assert send.numel() == recv.numel() * self.world and send.is_contiguous() and recv.is_contiguous()
        self._check(_fn("ddl_comm_reduce_scatter")(self._h, send.data_ptr(), recv.data_ptr(), recv.numel(),
                                                   _DTYPES[send.dtype], int(average), _stream()), "reduce_scatter")
        return self.collectives_launched if recv.numel() > 0 else 0

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor) -> int:
        """``recv`` = every rank's ``send`` in rank order (in place when ``send`` is
        ``recv``'s own rank slice); async, returns its sequence number."""
        assert recv.numel() == send.numel() * self.world and send.is_contiguous() and recv.is_contiguous()
        self._check(_fn("ddl_comm_all_gather")(self._h, send.data_ptr(), recv.data_ptr(), send.numel(),
                                               _DTYPES[send.dtype], _stream()), "all_gather")
        return self.collectives_launched if send.numel() > 0 else 0

    def wait(self) -> None:
        """Current (compute) stream waits for every collective issued so far."""
        self._check(_fn("ddl_comm_wait")(self._h, _stream()), "wait")

    def synchronize(self) -> None:
        self._check(_fn("ddl_comm_synchronize")(self._h), "synchronize")

    @property
    def collectives_launched(self) -> int:
        return int(_fn("ddl_comm_stats")(self._h, 0))

    def close(self, abort: bool = False) -> None:
        """Destroy the communicator.  ``abort=True`` (``ncclCommAbort``) is the failure
        path: it returns without waiting for peers and unblocks collectives stuck on a
        rank that died, so this rank can raise instead of hanging until the timeout."""
        wd = getattr(self, "watchdog", None)
        if wd is not None:
            wd.stop()
            self.watchdog = None
        if getattr(self, "_h", None):
            _fn("ddl_comm_destroy")(self._h, int(abort or bool(getattr(self, "failed", None))))
            self._h = None
        if _ACTIVE is self:
            set_active(None)

    # no __del__: destroying a communicator during interpreter teardown can block
    # on peers that already exited; process exit releases it.


# ---------------------------------------------------------------------- bucket policy
class TorchCollectives:
    """The ``all_reduce(t)`` / ``wait()`` contract of :func:`probe_allreduce` over a plain
    ``torch.distributed`` group: the auto bucket policy's probe where the native engine is not
    used (gloo on the CPU, or ``comm="torch"`` on GPUs)."""

    def __init__(self, group=None):
        self.group = group

    def all_reduce(self, t: torch.Tensor) -> int:
        dist.all_reduce(t, group=self.group)
        return 0

    def wait(self) -> None:
        pass


def probe_allreduce(engine, device, sizes_mb: Sequence[float] = (1, 4, 16, 64), iters: int = 5,
                    dtype: torch.dtype = torch.bfloat16, world: Optional[int] = None,
                    agree: bool = True) -> List[Dict[str, float]]:
    """Time all-reduces of each size on ``engine`` (``all_reduce(t)`` + ``wait()``: the native
    engine, or any stand-in with that contract): one warm-up, then the median of ``iters``
    host-timed calls with the device synchronised around each.  Returns per size: MB, ms,
    algorithm bandwidth (GB/s = bytes / t) and bus bandwidth (x 2(n-1)/n, the per-link figure
    of a ring: comparable across world sizes).  Every rank must call it (collective).

    ``agree``: each size's time is the MAX over the world's ranks (one scalar all-reduce), so every
    rank derives the same bucket layout from the probe -- per-rank host timings differ, and ranks
    whose buckets differ would issue all-reduces of different sizes against each other."""
    from . import dist as ddist
    n = int(world if world is not None else dist.get_world_size())
    esz = torch.empty((), dtype=dtype).element_size()
    sync = torch.cuda.synchronize if torch.device(device).type == "cuda" else (lambda: None)
    rows = []
    for mb in sizes_mb:
        t = torch.ones(max(1, int(mb * (1 << 20)) // esz), dtype=dtype, device=device)
        times = []
        for i in range(iters + 1):
            sync()
            t0 = time.perf_counter()
            engine.all_reduce(t)
            engine.wait()
            sync()
            if i:
                times.append(time.perf_counter() - t0)
        rows.append((float(mb), 1e3 * sorted(times)[len(times) // 2], t.numel() * esz))
    ms_all = [r[1] for r in rows]
    if agree and n > 1 and dist.is_available() and dist.is_initialized():
        ms_all = ddist.all_reduce_scalars(ms_all, op="max")
    out = []
    for (mb, _, nbytes), ms in zip(rows, ms_all):
        ms = round(ms, 4)
        alg = nbytes / (max(ms, 1e-6) * 1e-3) / 1e9
        out.append({"mb": mb, "ms": ms, "algbw_gbs": round(alg, 2),
                    "busbw_gbs": round(alg * 2 * (n - 1) / max(n, 1), 2)})
    return out


def fit_latency_bandwidth(probe: Sequence[Dict[str, float]]) -> Tuple[float, float]:
    """Least-squares fit of ``t = alpha + bytes / beta`` over the probe points: (alpha in ms,
    beta in bytes per ms).  A degenerate fit falls back to the largest message's rate."""
    xs = [p["mb"] * (1 << 20) for p in probe]
    ys = [p["ms"] for p in probe]
    k = len(xs)
    mx, my = sum(xs) / k, sum(ys) / k
    sxx = sum((x - mx) ** 2 for x in xs)
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx if sxx > 0 else 0.0
    if slope <= 0:
        big = max(range(k), key=lambda i: xs[i])
        return 0.0, xs[big] / max(ys[big], 1e-9)
    return max(0.0, my - slope * mx), 1.0 / slope


def auto_buckets(probe: Sequence[Dict[str, float]], total_mb: float) -> Tuple[float, float]:
    """(first_bucket_mb, bucket_mb) from a probe.

    A bucket of S bytes costs alpha + S / beta on the wire; its fixed part alpha is pure
    overhead, which stays under ~1/8 of the bucket's time once S >= 8 alpha beta.  So
    ``bucket_mb`` = 8 alpha beta, clamped to [4, 64] MB and to a quarter of the gradient (at
    least four buckets to overlap with backward); the first bucket -- the one the backward's
    first layers fill while every later bucket is still being computed -- is
    max(1 MB, 2 alpha beta), at most half a bucket, so the first ring starts early."""
    alpha, beta = fit_latency_bandwidth(probe)
    knee_mb = alpha * beta / (1 << 20)
    bucket = min(64.0, max(4.0, 8.0 * knee_mb), max(4.0, total_mb / 4.0))
    first = min(bucket / 2.0, max(1.0, 2.0 * knee_mb))
    return round(first, 2), round(bucket, 2)
