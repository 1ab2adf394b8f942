# Databricks notebook source
# MAGIC %md
# MAGIC ## ResNet-50 export + inference runtime comparison on MI355X
# MAGIC
# MAGIC Same experiment as the reference notebook (`notebooks/cv/onnx_experiments.py` of
# MAGIC rafaelvp-db/databricks-distributed-deep-learning): export ResNet-50, run it on several
# MAGIC runtimes, print top-5, check parity, compare artifact sizes. Runtimes here: PyTorch eager
# MAGIC fp32 (oracle), TorchScript, the framework's native bf16 HIP kernels, and the native
# MAGIC inference graph (BN folded, conv+bias+residual+ReLU fused, replayed from a hipGraph).
# MAGIC Random-init weights (no network for pretrained weights) and a synthetic image.

# COMMAND ----------

import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__) if "__file__" in dir() else ".", "../..")))

import torch

from databricks_distributed_deep_learning_amd.data import imagenet_preprocess
from databricks_distributed_deep_learning_amd.export import bench_runtimes
from databricks_distributed_deep_learning_amd.models import resnet50

SMOKE = os.environ.get("DDL_NOTEBOOK_SMOKE") == "1"

# COMMAND ----------

# DBTITLE 1,Model + preprocessed input (synthetic 480x640 RGB "photo")
torch.manual_seed(0)
model = resnet50().eval()
img = (torch.rand(480, 640, 3) * 255).to(torch.uint8).numpy()
x = imagenet_preprocess(img).unsqueeze(0).permute(0, 2, 3, 1).contiguous()   # NHWC batch of 1
device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
print("GPU Availability:", torch.cuda.is_available())

# COMMAND ----------

# DBTITLE 1,Runtime comparison, parity and artifact sizes
report = bench_runtimes(model.to(device), x.to(device), iters=2 if SMOKE else 50, warmup=1 if SMOKE else 5)
for name, r in report["runtimes"].items():
    print(f"{name:32s} {r['ms']:8.2f} ms  top1={r['top5'][0]}  "
          + (f"max_abs_err={r['max_abs_err']:.3e} top1_agrees={r['top1_agrees']}" if "max_abs_err" in r else ""))
print(json.dumps(report["artifact_bytes"], indent=1))
