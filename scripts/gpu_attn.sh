# attention / dropout / LN tests, attention microbench (fused vs two-kernel backward), bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1; rc=$?; tail -2 gpurun_out/t_attn.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_attn.log | head; exit $rc; }
timeout -k 10 300 python benchmarks/attention_bench.py > gpurun_out/attn_bench.log 2>&1 || { tail -20 gpurun_out/attn_bench.log; exit 1; }
grep shape gpurun_out/attn_bench.log
DDL_ATTN_FUSED_BWD=0 timeout -k 10 300 python benchmarks/attention_bench.py --shapes bert_base > gpurun_out/attn_bench_twokernel.log 2>&1 || exit 1
echo "== two-kernel backward"; grep shape gpurun_out/attn_bench_twokernel.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
