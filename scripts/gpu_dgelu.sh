set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_models_gpu.py tests/test_fusions_gpu.py tests/test_export_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_dgelu.log 2>&1; rc=$?
tail -2 gpurun_out/test_dgelu.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/test_dgelu.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 20 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
