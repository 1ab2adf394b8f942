#!/bin/bash
# GELU-epilogue A/B: GEMM microbenchmark + BERT bench, current library vs the "base" variant.
set -o pipefail
mkdir -p gpurun_out
for arm in cur base cur base; do
  if [ $arm = cur ]; then unset DDL_NATIVE_LIB; else export DDL_NATIVE_LIB=$PWD/databricks_distributed_deep_learning_amd/_native/ab/libddl_base.so; fi
  timeout -k 10 200 python benchmarks/comm_overlap.py --occupy 0 > gpurun_out/gelu_mb_$arm.log 2>&1 || exit $?
  echo "$arm micro: $(grep -o '"shape": "bert_[a-z0-9_]*gelu[a-z_]*".*"alone_ms": [0-9.]*' gpurun_out/gelu_mb_$arm.log | sed 's/"M".*"alone_ms"//' | tr '\n' ' ')"
done
bash scripts/gpu_ab_bert.sh base 2
