# Bias preload / dGELU batched loads / store-behind mask: tests, per-GEMM traces and bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_fusions_gpu.py tests/test_models_gpu.py tests/test_race_screen_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_behind.log 2>&1 || { tail -30 gpurun_out/test_behind.log; exit 1; }
tail -1 gpurun_out/test_behind.log
for m in 0 3 0 3; do
  DDL_GEMM_BEHIND=$m timeout -k 10 300 python scripts/debug/gemm_trace.py bert_base --top 12 > gpurun_out/gemm_trace_bert_b$m.md 2> gpurun_out/gemm_trace_bert.err || { tail -20 gpurun_out/gemm_trace_bert.err; exit 1; }
  echo "== behind=$m"; sed -n 6,20p gpurun_out/gemm_trace_bert_b$m.md
done
for m in 0 3 0 3; do
  DDL_GEMM_BEHIND=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_b$m.log 2>&1 || { tail -20 gpurun_out/bench_b$m.log; exit 1; }
  echo "behind=$m $(tail -1 gpurun_out/bench_b$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["bert_base_samples_per_sec"])')"
done
