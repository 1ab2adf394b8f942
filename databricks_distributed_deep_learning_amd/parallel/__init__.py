"""Distributed runtime: process groups, launchers, the RCCL gradient reducer."""
from . import dist  # noqa: F401
from .dist import (init, destroy, rank, world_size, local_rank, is_main, barrier,  # noqa: F401
                   all_reduce_scalars, all_gather_object, broadcast_object, broadcast_tensors, device)
from .ddp import DataParallel, ReplicaDivergence  # noqa: F401
from .launcher import Distributor, TorchDistributor, ChildFailed  # noqa: F401
from .horovod import HorovodRunner  # noqa: F401
from . import horovod as hvd  # noqa: F401
