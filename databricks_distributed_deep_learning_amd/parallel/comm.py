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
"""
from __future__ import annotations

import ctypes
import glob
import os
from typing import Optional, Sequence

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


class NativeComm:
    """RCCL communicator over all ranks of ``group`` (default: the world)."""

    def __init__(self, group=None, device: Optional[torch.device] = None):
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

    # ------------------------------------------------------------------
    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise CommError(f"{what} failed ({rc}): {_err()}")

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
        if getattr(self, "_h", None):
            _fn("ddl_comm_destroy")(self._h, int(abort))
            self._h = None
        if _ACTIVE is self:
            set_active(None)

    # no __del__: destroying a communicator during interpreter teardown can block
    # on peers that already exited; process exit releases it.
