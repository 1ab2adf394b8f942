"""Throughput meter, device timers and rank-0 JSONL metrics.

The reference times one sample with ``time.time()`` and no warm-up or device
sync (``notebooks/cv/onnx_experiments.py:92-104,133-140``); here timing is
bracketed by device synchronisation, warm-up is excluded, and results are
aggregated across ranks.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import torch


def sync(device: Optional[torch.device] = None) -> None:
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)
    elif device is None and torch.cuda.is_available():
        torch.cuda.synchronize()


class StepTimer:
    """Host wall clock bracketed by device synchronisation."""

    def __init__(self, device: torch.device):
        self.device = device
        self.t0 = 0.0

    def start(self) -> None:
        sync(self.device)
        self.t0 = time.perf_counter()

    def stop(self) -> float:
        sync(self.device)
        return time.perf_counter() - self.t0


class EventTimer:
    """HIP-event timer for a region on the current stream (no host sync inside)."""

    def __init__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.b = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.a.record()
        return self

    def __exit__(self, *exc):
        self.b.record()

    def ms(self) -> float:
        self.b.synchronize()
        return self.a.elapsed_time(self.b)


class PhaseTimer:
    """Per-phase step-time breakdown (fwd / bwd / comm_wait / opt).

    ``mark(name)`` closes the phase that ran since the previous mark.  On the GPU a
    mark is one HIP event recorded on the compute stream (no host sync, so the timed
    loop is not perturbed); the events are resolved only in :meth:`summary`, at log
    points.  ``comm_wait`` is what the compute stream spent waiting for the last
    gradient all-reduces after its own backward work -- the EXPOSED communication.
    On the CPU marks are host clock readings."""

    def __init__(self, device: torch.device, enabled: bool = True, max_pending: int = 64):
        self.cuda = device.type == "cuda"
        self.enabled = enabled
        # steps whose marks may wait for summary(); beyond it end_step() folds the oldest
        # FINISHED steps into the totals (an event query, never a sync) and recycles their
        # events, so a long run without log points keeps a bounded event / host footprint
        self.max_pending = max(1, int(max_pending))
        self._pending: list = []       # per step: [(name, event or time), ...]
        self._cur: list = []
        self._pool: list = []          # resolved events, re-recorded by later marks
        self.totals: Dict[str, float] = {}
        self.steps = 0

    def _stamp(self):
        if self.cuda:
            e = self._pool.pop() if self._pool else torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def begin(self) -> None:
        if self.enabled:
            self._cur = [("", self._stamp())]

    def mark(self, name: str) -> None:
        if self.enabled and self._cur:
            self._cur.append((name, self._stamp()))

    def end_step(self) -> None:
        if self.enabled and len(self._cur) > 1:
            self._pending.append(self._cur)
            if len(self._pending) > self.max_pending:
                self._resolve(only_finished=True)
        self._cur = []

    def _fold(self, marks) -> None:
        for (_, a), (name, b) in zip(marks[:-1], marks[1:]):
            if self.cuda:
                b.synchronize()
                ms = a.elapsed_time(b)
            else:
                ms = 1000.0 * (b - a)
            self.totals[name] = self.totals.get(name, 0.0) + ms
        if self.cuda:
            self._pool.extend(e for _, e in marks)
        self.steps += 1

    def _resolve(self, only_finished: bool = False) -> None:
        """Fold pending steps into the totals, oldest first; ``only_finished``: stop at the
        first step whose last event has not completed (no host wait)."""
        n = 0
        for marks in self._pending:
            if only_finished and self.cuda and not marks[-1][1].query():
                break
            self._fold(marks)
            n += 1
        self._pending = self._pending[n:]

    def summary(self, reset: bool = False) -> Dict[str, float]:
        """Mean milliseconds per step of each phase since the last reset."""
        self._resolve()
        out = {f"{k}_ms": v / max(1, self.steps) for k, v in self.totals.items()}
        if reset:
            self.totals, self.steps = {}, 0
        return out


class ThroughputMeter:
    def __init__(self, items_per_step: int):
        self.items_per_step = items_per_step
        self.steps = 0
        self.seconds = 0.0

    def update(self, seconds: float, steps: int = 1) -> None:
        self.steps += steps
        self.seconds += seconds

    @property
    def items_per_sec(self) -> float:
        return self.items_per_step * self.steps / self.seconds if self.seconds > 0 else 0.0

    @property
    def ms_per_step(self) -> float:
        return 1000.0 * self.seconds / self.steps if self.steps else 0.0


def _mlflow_module(flag: Optional[bool]):
    """``mlflow`` when requested (``flag`` or DDL_MLFLOW=1) and importable, else None:
    the Databricks-native tracking sink, absent from this image, so strictly optional."""
    if flag is None:
        flag = os.environ.get("DDL_MLFLOW", "0") == "1"
    if not flag:
        return None
    try:
        import mlflow
    except ImportError:
        return None
    return mlflow


class JsonlLogger:
    """Rank-0 structured log: one JSON object per record; numeric fields
    are mirrored to MLflow (``log_metrics(step=record["step"])``) when enabled."""

    def __init__(self, path: str = "", enabled: bool = True, mlflow: Optional[bool] = None):
        self.path = path
        self.enabled = enabled and bool(path)
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._mlflow = _mlflow_module(mlflow) if enabled else None

    def log(self, record: Dict) -> None:
        if self._mlflow is not None:
            nums = {k: float(v) for k, v in record.items()
                    if isinstance(v, (int, float)) and not isinstance(v, bool) and k != "step"}
            if nums:
                self._mlflow.log_metrics(nums, step=int(record.get("step", 0)))
        if not self.enabled:
            return
        record = dict(record, ts=time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(record) + "\n")


def memory_stats(device: torch.device) -> Dict[str, float]:
    if device.type != "cuda":
        return {}
    return {"mem_alloc_gb": torch.cuda.memory_allocated(device) / 2**30,
            "mem_peak_gb": torch.cuda.max_memory_allocated(device) / 2**30}
