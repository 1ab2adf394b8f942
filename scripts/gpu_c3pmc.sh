#!/bin/bash
# hardware counters for the direct 3x3 conv kernels
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_c3
bash scripts/pmc_profile.sh gpurun_out/pmc_c3 -- python3 benchmarks/conv3x3_bench.py --grid 0 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_c3 --match conv3x3 > gpurun_out/pmc_c3.md
rm -rf gpurun_out/pmc_c3
cat gpurun_out/pmc_c3.md
