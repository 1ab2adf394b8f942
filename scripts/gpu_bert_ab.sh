set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_attention_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_bert.log 2>&1 || { tail -30 gpurun_out/test_bert.log; exit 1; }
tail -2 gpurun_out/test_bert.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python3 bench.py --model bert_base --steps 5 --warmup 3 > gpurun_out/prof_bert.log 2>&1 || exit $?
tail -1 gpurun_out/prof_bert.log | cut -c1-160
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
