"""Attribute small ATen kernels (copies, fills, adds) in one training step to ops (GPU debugging aid)."""
import sys

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.config import get_preset  # noqa: E402
from databricks_distributed_deep_learning_amd.training.loop import Trainer  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
cfg = get_preset("resnet50_ddp" if model == "resnet50" else "bert_base_ddp", steps=1, warmup_steps=1, log_every=0)
tr = Trainer(cfg)
for _ in range(2):
    tr.train_step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    tr.train_step()
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ka if e.key in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add_", "aten::add",
                                   "aten::index", "aten::flip", "aten::clone", "aten::zeros", "aten::to",
                                   "aten::_to_copy", "aten::contiguous")]
rows.sort(key=lambda e: -e.count)
for e in rows[:40]:
    print(f"{e.key:20s} n={e.count:4d} dev_us={e.self_device_time_total:9.1f}")
    for fr in (e.stack or [])[:6]:
        print("      ", fr)
