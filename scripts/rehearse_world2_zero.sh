#!/bin/bash
# 2-rank rehearsal on ONE GPU (gloo) of the sharded-optimizer and SyncBatchNorm paths
# with the native kernels: ZeRO-1 slices, LAMB/AdamW/SGD phase split, all-gathers.
set -o pipefail
mkdir -p gpurun_out
export DDL_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --bert-batch 32 --zero --sync-bn
