#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 ranks share cuda:0 over gloo (RCCL refuses
# two ranks on one device).  Exercises the bucketed reducer with GPU tensors,
# the HIP kernels' direct-to-arena weight gradients + bucket hooks, per-rank
# data, max-over-ranks timing and the bench JSON contract at world size 2.
set -o pipefail
mkdir -p gpurun_out
export DDL_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --bert-batch 32
