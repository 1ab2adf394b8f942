"""Test-only fault injection.

``maybe_fail(step, cfg)`` raises :class:`InjectedFault` on rank ``cfg.fault_rank``
at step ``cfg.fault_step`` (or ``DDL_FAULT_RANK`` / ``DDL_FAULT_STEP`` env vars),
so the launcher's first-failure propagation and sibling teardown can be tested.
"""
from __future__ import annotations

import os

from ..parallel import dist as ddist


class InjectedFault(RuntimeError):
    pass


def maybe_fail(step: int, fault_rank: int = -1, fault_step: int = -1) -> None:
    fr = int(os.environ.get("DDL_FAULT_RANK", fault_rank))
    fs = int(os.environ.get("DDL_FAULT_STEP", fault_step))
    if fr >= 0 and fs >= 0 and ddist.rank() == fr and step == fs:
        raise InjectedFault(f"injected fault on rank {fr} at step {fs}")
