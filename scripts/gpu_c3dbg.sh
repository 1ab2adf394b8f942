#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 4 3 7; do
  DDL_CONV3X3_DBG=$d timeout -k 10 120 python benchmarks/conv3x3_bench.py --grid 0 > gpurun_out/c3dbg_$d.log 2>&1 || exit $?
  echo "dbg=$d $(grep direct gpurun_out/c3dbg_$d.log | tr '\n' ' ')"
done
