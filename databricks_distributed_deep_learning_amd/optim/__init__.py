"""Optimizers over a flat parameter arena (fp32 master weights)."""
from .arena import ParamArena  # noqa: F401
from .flat import FlatSGD, FlatAdamW, FlatLAMB, FlatOptimizer, build_optimizer, LRSchedule  # noqa: F401
