"""roctx ranges + rocprofv3 command builder (north-star N10).

``range("fwd")`` pushes a roctx range (visible in ``rocprofv3 --marker-trace``)
when ``libroctx64`` is loadable, and is a no-op otherwise.
``rocprof_cmd`` builds the pool-safe profiling commands: kernel trace + stats in
one run, PMC counters in a separate run (never combined with sys/runtime trace).
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os
from typing import List, Optional, Sequence

_roctx = None
_tried = False


def _lib():
    global _roctx, _tried
    if not _tried:
        _tried = True
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                _roctx = ctypes.CDLL(name)
                _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
    return _roctx


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _lib() if os.environ.get("DDL_ROCTX", "0") == "1" else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


# PMC sets that fit gfx950 slot limits (SQ 8, TCC 4 — FETCH_SIZE and WRITE_SIZE not together)
PMC_SETS = {
    "mfma": ["SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
    "lds": ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_LDS"],
    "hbm_read": ["FETCH_SIZE", "GRBM_GUI_ACTIVE"],
    "hbm_write": ["WRITE_SIZE", "GRBM_GUI_ACTIVE"],
}


def rocprof_cmd(cmd: Sequence[str], out_dir: str, pmc: Optional[str] = None) -> List[str]:
    base = ["rocprofv3", "--output-format", "csv", "-d", out_dir]
    if pmc:
        return base + ["--kernel-trace", "--pmc", *PMC_SETS[pmc], "--"] + list(cmd)
    return base + ["--kernel-trace", "--stats", "--"] + list(cmd)
