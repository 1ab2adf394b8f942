# Residual-epilogue change: GEMM/fusion/model tests, per-GEMM trace, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_fusions_gpu.py tests/test_models_gpu.py tests/test_race_screen_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_res.log 2>&1 || { tail -30 gpurun_out/test_res.log; exit 1; }
tail -1 gpurun_out/test_res.log
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 45 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
grep -E "^1[0-9]+ GEMM|\| res \|" gpurun_out/gemm_trace_r50.md
timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/bench_res.log 2>&1 || { tail -20 gpurun_out/bench_res.log; exit 1; }
tail -1 gpurun_out/bench_res.log | cut -c1-200
