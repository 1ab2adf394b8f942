# Databricks notebook source
# MAGIC %md
# MAGIC ## ViT-B/16 bf16 training (shares the NLP attention / LayerNorm / GEMM kernels)

# COMMAND ----------

import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__) if "__file__" in dir() else ".", "../..")))

import torch

from databricks_distributed_deep_learning_amd import get_preset
from databricks_distributed_deep_learning_amd.parallel import Distributor
from databricks_distributed_deep_learning_amd.training import train

SMOKE = os.environ.get("DDL_NOTEBOOK_SMOKE") == "1"

# COMMAND ----------

if SMOKE or not torch.cuda.is_available():
    cfg = get_preset("vit_b16", batch_size=1, image_size=32, steps=1, warmup_steps=0, dtype="fp32",
                     backend="gloo", native="off", num_classes=10)
    n, gpu = 1, False
else:
    cfg = get_preset("vit_b16", steps=20, warmup_steps=3)
    n, gpu = torch.cuda.device_count(), True
if __name__ == "__main__":
    print(Distributor(num_processes=n, use_gpu=gpu).run(train, cfg))
