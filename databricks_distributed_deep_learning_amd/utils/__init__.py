"""Utilities: metrics/timers, checkpointing, profiling, fault injection, memory sizing."""
from . import metrics, checkpoint, profiling, faults, memory  # noqa: F401
