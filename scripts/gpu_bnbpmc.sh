#!/bin/bash
# hardware counters for the BN-backward dgrad GEMM epilogue microbenchmark
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_bnb
bash scripts/pmc_profile.sh gpurun_out/pmc_bnb -- python3 benchmarks/bnb_gemm_bench.py || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_bnb --match gemm > gpurun_out/pmc_bnb.md
rm -rf gpurun_out/pmc_bnb
cat gpurun_out/pmc_bnb.md
