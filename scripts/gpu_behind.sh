set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_fusions_gpu.py tests/test_models_gpu.py tests/test_race_screen_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_behind.log 2>&1; rc=$?
tail -2 gpurun_out/test_behind.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/test_behind.log | head -20; exit $rc; }
timeout -k 10 120 build/gemm_sweep big 0 802816 256 64 1 bigs 0 802816 256 64 1 big 0 200704 512 128 1 big 0 50176 1024 256 1 big 0 16384 3072 768 1 > gpurun_out/behind_sweep.log 2>&1 && cat gpurun_out/behind_sweep.log
DDL_GEMM_DIRECT=0 timeout -k 10 120 build/gemm_sweep big 0 802816 256 64 1 big 0 200704 512 128 1 big 0 50176 1024 256 1 > gpurun_out/behind_sweep0.log 2>&1 && cat gpurun_out/behind_sweep0.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
