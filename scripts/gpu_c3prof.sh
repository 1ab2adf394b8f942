#!/bin/bash
# kernel-level timing of the direct 3x3 conv (rocprofv3 kernel trace), per debug mode and grid
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in ${DBGS:-0}; do
  for g in ${GRIDS:-0}; do
    DDL_CONV3X3_DBG=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof_${d}_$g -o run -- python3 benchmarks/conv3x3_bench.py --grid $g > gpurun_out/c3prof_${d}_$g.log 2>&1 || exit $?
    echo "dbg=$d grid=$g $(python3 scripts/prof_summary.py gpurun_out/c3prof_${d}_$g/run_results.db --steps 1 --names x --top 12 | grep conv3x3 | tr '\n' ' ')"
    rm -rf gpurun_out/c3prof_${d}_$g
  done
done
