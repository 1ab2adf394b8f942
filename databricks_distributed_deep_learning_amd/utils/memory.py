"""HBM-aware batch sizing (north-star N13, BASELINE.json:11 "288 GB HBM batch sizing").

``fit_batch_size`` probes: run one fwd+bwd at a candidate micro-batch, read the
peak allocation, extrapolate linearly (activation memory is linear in batch),
and back off on OOM, keeping ``headroom`` of the device free.  Everything is
sized for one MI355X's 288 GB.
"""
from __future__ import annotations

from typing import Any, Callable, Dict

import torch

# the last fit's decisions (reported in the training summary as ``auto_batch``)
last_fit: Dict[str, Any] = {}


def fit_batch_size(step_fn: Callable[[int], None], device: torch.device, start: int = 8,
                   max_batch: int = 4096, headroom: float = 0.15, multiple: int = 8) -> int:
    if device.type != "cuda":
        return start
    total = torch.cuda.get_device_properties(device).total_memory
    budget = total * (1.0 - headroom)

    def peak_at(b: int) -> float:
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(device)
        base = torch.cuda.memory_allocated(device)
        step_fn(b)
        torch.cuda.synchronize(device)
        peak = torch.cuda.max_memory_allocated(device) - base
        last_fit["probes"].append([b, round(peak / 2**30, 2)])
        return peak

    last_fit.clear()
    last_fit.update(budget_gb=round(budget / 2**30, 2), probes=[])
    b0 = start
    while True:
        try:
            p0 = peak_at(b0)
            break
        except torch.cuda.OutOfMemoryError:
            b0 //= 2
            if b0 < 1:
                raise
    static = torch.cuda.memory_allocated(device)
    per_sample = p0 / b0
    last_fit.update(static_gb=round(static / 2**30, 2), gb_per_sample=round(per_sample / 2**30, 4))
    est = int((budget - static) / max(per_sample, 1.0))
    est = max(b0, min(max_batch, est // multiple * multiple))
    # the candidate must FIT THE BUDGET, not merely run: a probe that squeezed into the last few GB
    # left nothing for what the probe step does not do (optimizer scratch, the fp32 accumulation
    # arena, GEMM tuning workspaces at an untuned batch) -- BERT-large LAMB went out of memory in its
    # first real step that way (round 6).  Over budget: shrink in proportion and probe again.
    while est > b0:
        try:
            p = peak_at(est)
        except torch.cuda.OutOfMemoryError:
            est = max(b0, int(est * 0.8) // multiple * multiple)
            last_fit["probes"].append([est, "oom"])
            continue
        if static + p <= budget:
            last_fit["batch"] = est
            return est
        est = max(b0, min(est - multiple, int(est * (budget - static) / p)) // multiple * multiple)
    last_fit["batch"] = b0
    return b0
