# Databricks notebook source
# MAGIC %md
# MAGIC ## ResNet-50 data-parallel training on one 8x MI355X node
# MAGIC
# MAGIC TorchDistributor-style launch: `Distributor(num_processes=8).run(train, cfg)` starts one
# MAGIC process per GPU; gradients are all-reduced in buckets over RCCL/xGMI while backward runs.
# MAGIC Data: synthetic ImageNet-shape batches (replaces the Petastorm/Delta reader).

# COMMAND ----------

import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__) if "__file__" in dir() else ".", "../..")))

import torch

from databricks_distributed_deep_learning_amd import get_preset
from databricks_distributed_deep_learning_amd.parallel import Distributor
from databricks_distributed_deep_learning_amd.training import train

SMOKE = os.environ.get("DDL_NOTEBOOK_SMOKE") == "1"          # CPU / gloo, 2 ranks
GPU_SMOKE = os.environ.get("DDL_NOTEBOOK_SMOKE") == "gpu"    # the GPU branch, a few small steps

# COMMAND ----------

# DBTITLE 1,Configuration
if SMOKE or not torch.cuda.is_available():
    cfg = get_preset("resnet18_gloo", batch_size=2, image_size=32, steps=2, warmup_steps=1, num_classes=10)
    nproc, use_gpu = 2, False
else:
    cfg = get_preset("resnet50_ddp", steps=50, warmup_steps=5)
    if GPU_SMOKE:
        cfg = cfg.replace(batch_size=32, steps=3, warmup_steps=1, log_every=1)
    nproc, use_gpu = torch.cuda.device_count(), True
print(cfg)

# COMMAND ----------

# DBTITLE 1,Launch
if __name__ == "__main__":   # spawned ranks re-import this file; only the driver launches
    summary = Distributor(num_processes=nproc, local_mode=True, use_gpu=use_gpu).run(train, cfg)
    print(summary)
