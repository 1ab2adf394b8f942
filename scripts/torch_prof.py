#!/usr/bin/env python3
"""Which Python ops launch the non-native (at::native) kernels of a training step:
    python scripts/torch_prof.py [resnet50|bert_base] > gpurun_out/torch_prof.txt
torch.profiler over two steady-state steps, the at:: kernels grouped by their Python stack."""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.config import get_preset  # noqa: E402
from databricks_distributed_deep_learning_amd.parallel import dist as ddist  # noqa: E402
from databricks_distributed_deep_learning_amd.training.loop import Trainer  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "bert_base"
ddist.init("auto")
cfg = get_preset("resnet50_ddp" if model == "resnet50" else "bert_base_ddp",
                 batch_size=256 if model == "resnet50" else 128, **({} if model == "resnet50" else {"dropout": 0.1}))
cfg = cfg.replace(log_every=0)
tr = Trainer(cfg)
for _ in range(4):
    tr.train_step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for _ in range(2):
        tr.train_step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=60,
                                                   max_src_column_width=200))

# where each ATen op that launched device work comes from (first frames inside this package)
from collections import defaultdict  # noqa: E402

agg = defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if not ev.name.startswith("aten::") or ev.device_time_total <= 0:
        continue
    frames = [f for f in (ev.stack or []) if "databricks_distributed" in f][:3]
    key = (ev.name, " <- ".join(f.split("databricks_distributed_deep_learning_amd/")[-1] for f in frames))
    agg[key][0] += 1
    agg[key][1] += ev.device_time_total
print("\n### ATen ops with device time, by call site (2 steps)")
for (name, where), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{us:9.1f} us {n:4d}x {name:28s} {where}")
