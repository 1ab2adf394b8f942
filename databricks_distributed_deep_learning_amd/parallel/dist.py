"""Process-group bootstrap and collective helpers (north-star component N5).

The reference has no distributed code at all; this module is the
MI355X-native replacement for what HorovodRunner / TorchDistributor set up on a
Databricks cluster.  Topology: one process per GPU on one node, RCCL (the
``"nccl"`` backend of PyTorch-ROCm) over xGMI for GPU tensors, gloo for the CPU
plumbing tests (BASELINE.json:7).
"""
from __future__ import annotations

import datetime
import os
from typing import Any, List, Optional

import torch
import torch.distributed as dist

_DEVICE: Optional[torch.device] = None


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else env_int("RANK", 0)


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else env_int("WORLD_SIZE", 1)


def local_rank() -> int:
    return env_int("LOCAL_RANK", rank())


def is_main() -> bool:
    return rank() == 0


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def gpu_available() -> bool:
    # device_count() does not initialise the GPU on this image; is_available() does.
    return torch.cuda.is_available()


def resolve_backend(backend: str = "auto", use_gpu: Optional[bool] = None) -> str:
    if backend not in ("auto", None):
        return backend
    if use_gpu is None:
        use_gpu = gpu_available()
    return "nccl" if use_gpu else "gloo"


def device() -> torch.device:
    global _DEVICE
    if _DEVICE is None:
        if gpu_available():
            _DEVICE = torch.device("cuda", local_rank() % max(1, torch.cuda.device_count()))
        else:
            _DEVICE = torch.device("cpu")
    return _DEVICE


def init(backend: str = "auto", timeout_s: float = 600.0, use_gpu: Optional[bool] = None) -> None:
    """Initialise the default process group from torchrun-style env vars.

    Safe to call when WORLD_SIZE is unset/1 (creates a 1-rank group so the same
    code path runs in a notebook), and idempotent.
    """
    global _DEVICE
    if is_initialized():
        return
    backend = resolve_backend(backend, use_gpu)
    if use_gpu is None:
        use_gpu = gpu_available()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", os.environ["RANK"])
    # dmabuf IPC only on this pool (see task environment notes).
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    kw = {}
    if backend == "nccl":
        lr = local_rank()
        torch.cuda.set_device(lr)
        _DEVICE = torch.device("cuda", lr)
        kw["device_id"] = _DEVICE
    else:
        # gloo with GPU tensors (e.g. several ranks sharing one GPU in a rehearsal)
        _DEVICE = torch.device("cuda", local_rank() % max(1, torch.cuda.device_count())) \
            if (use_gpu and gpu_available()) else torch.device("cpu")
    dist.init_process_group(backend=backend, init_method="env://",
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)


def destroy() -> None:
    global _DEVICE
    if is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()
    _DEVICE = None


def barrier() -> None:
    if is_initialized() and world_size() > 1:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def _comm_device() -> torch.device:
    if is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_scalars(values: List[float], op: str = "sum") -> List[float]:
    """Metric all-reduce (collective C4): a handful of scalars, latency-bound."""
    if not is_initialized() or world_size() == 1:
        return list(values)
    t = torch.tensor(values, dtype=torch.float64 if _comm_device().type == "cpu" else torch.float32,
                     device=_comm_device())
    rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
    dist.all_reduce(t, op=rop)
    return [float(v) for v in t.tolist()]


def all_gather_object(obj: Any) -> List[Any]:
    """All-gather of small python objects (collective C6)."""
    if not is_initialized() or world_size() == 1:
        return [obj]
    out: List[Any] = [None] * world_size()
    dist.all_gather_object(out, obj)
    return out


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not is_initialized() or world_size() == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


@torch.no_grad()
def broadcast_tensors(tensors, src: int = 0, bucket_bytes: int = 256 << 20) -> None:
    """Broadcast params/buffers from ``src`` (collective C1), flattened into large
    buckets so the xGMI ring moves few, big messages instead of 161 tiny ones."""
    if not is_initialized() or world_size() == 1:
        return
    tensors = [t for t in tensors if t.numel() > 0]
    groups = {}
    for t in tensors:
        groups.setdefault((t.dtype, t.device), []).append(t)
    for (_, _dev), ts in groups.items():
        cur, cur_bytes = [], 0
        for t in ts + [None]:
            if t is not None and cur_bytes + t.numel() * t.element_size() <= bucket_bytes:
                cur.append(t)
                cur_bytes += t.numel() * t.element_size()
                continue
            if cur:
                flat = torch.cat([c.reshape(-1) for c in cur])
                dist.broadcast(flat, src=src)
                off = 0
                for c in cur:
                    n = c.numel()
                    c.copy_(flat[off:off + n].view_as(c))
                    off += n
            cur, cur_bytes = ([t], t.numel() * t.element_size()) if t is not None else ([], 0)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


free_port = _free_port
