# Databricks notebook source
# MAGIC %md
# MAGIC ## BERT-large seq 512 with LAMB, gradient accumulation and HBM-aware batch sizing
# MAGIC
# MAGIC `batch_size=0` asks the trainer to size the micro-batch for the 288 GB of one MI355X
# MAGIC (probe one fwd+bwd, extrapolate, back off on OOM); `grad_accum` micro-steps run under
# MAGIC `no_sync()` with fp32 gradient accumulation, and the fused LAMB kernel applies per-tensor
# MAGIC trust ratios in one launch over the flat parameter arena.

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
    cfg = get_preset("bert_large_lamb", batch_size=1, seq_len=16, steps=1, warmup_steps=0, grad_accum=2,
                     dtype="fp32", backend="gloo", native="off")
    n, gpu = 1, False
else:
    cfg = get_preset("bert_large_lamb", steps=10, warmup_steps=2)
    n, gpu = torch.cuda.device_count(), True
if __name__ == "__main__":
    print(Distributor(num_processes=n, use_gpu=gpu).run(train, cfg))
