#!/usr/bin/env python3
"""Which framework call sites still dispatch device work to ATen in a training step.

    python scripts/debug/aten_sites.py [bert_base|resnet50|vit_b16|bert_large_lamb]

A TorchDispatchMode records every ATen op that touches a CUDA tensor during one steady-state step
(forward, backward, reducer, optimizer), with the innermost frames of this package on the Python
stack (autograd-engine ops carry the forward frame that recorded their node), grouped and counted.
Views and metadata ops (no kernel) are filtered out.
"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd.config import get_preset  # noqa: E402
from databricks_distributed_deep_learning_amd.parallel import dist as ddist  # noqa: E402
from databricks_distributed_deep_learning_amd.training.loop import Trainer  # noqa: E402

NO_KERNEL = ("view", "_unsafe_view", "reshape", "as_strided", "t", "transpose", "permute", "expand", "slice", "select",
             "unsqueeze", "squeeze", "detach", "alias", "empty", "empty_like", "empty_strided", "_reshape_alias",
             "split", "chunk", "narrow", "unbind", "lift_fresh", "resolve_conj", "resolve_neg", "_to_copy_noop",
             "is_same_size", "result_type", "_local_scalar_dense", "set_", "record_stream", "split_with_sizes",
             "new_empty", "new_empty_strided", "unflatten", "flatten", "contiguous")


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        name = func.overloadpacket.__name__
        if name in NO_KERNEL:
            return out
        tensors = [a for a in list(args) + list(kwargs.values()) if isinstance(a, torch.Tensor)]
        if isinstance(out, torch.Tensor):
            tensors.append(out)
        if not any(t.is_cuda for t in tensors):
            return out
        frames = [f for f in traceback.extract_stack()[:-1] if "databricks_distributed_deep_learning_amd" in f.filename]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(frames[-3:]))
        self.count[(name, where)] += 1
        return out


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "bert_base"
    ddist.init("auto")
    if model == "resnet50":
        cfg = get_preset("resnet50_ddp", batch_size=256)
    elif model == "vit_b16":
        cfg = get_preset("vit_b16")
    elif model == "bert_large_lamb":     # the profiled configuration (scripts/gpu.sh run_model)
        cfg = get_preset("bert_large_lamb", batch_size=32)
    else:
        cfg = get_preset("bert_base_ddp", batch_size=128, dropout=0.1)
    tr = Trainer(cfg.replace(log_every=0))
    for _ in range(3):
        tr.train_step()
    torch.cuda.synchronize()
    mode = Sites()
    with mode:
        tr.train_step()
    torch.cuda.synchronize()
    for (name, where), n in sorted(mode.count.items(), key=lambda kv: (-kv[1], kv[0])):
        print(f"{n:4d}  {name:24s} {where}")
    tr.close()


if __name__ == "__main__":
    main()
