# Quick ResNet-50 check: GEMM trace + bench (no tests).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 30 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
