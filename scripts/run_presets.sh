#!/bin/bash
# GPU smoke of every BASELINE preset through the notebook-style train() CLI
# (few steps each; prints one summary JSON line per preset).
set -o pipefail
mkdir -p gpurun_out
M=databricks_distributed_deep_learning_amd.training.loop
for spec in "resnet18_gloo:--backend=nccl --steps=3 --warmup_steps=1" \
            "resnet50_ddp:--steps=3 --warmup_steps=1" \
            "bert_base_ddp:--steps=3 --warmup_steps=1" \
            "vit_b16:--steps=3 --warmup_steps=1" \
            "bert_large_lamb:--steps=2 --warmup_steps=1"; do
  name="${spec%%:*}"; args="${spec#*:}"
  echo "=== $name $args" >&2
  timeout -k 10 400 python -m $M --preset $name $args > gpurun_out/preset_$name.log 2>&1
  rc=$?
  echo "=== $name rc=$rc" >&2
  tail -2 gpurun_out/preset_$name.log | cut -c1-600 >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
