# In-run A/B of the BN-backward dgrad epilogue (off / without residual dgrads / all) + GEMM trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_fusions_gpu.py -x -q -k "bn_backward or bn_stats" --timeout 120 --timeout-method thread > gpurun_out/test_bnb.log 2>&1 || { tail -30 gpurun_out/test_bnb.log; exit 1; }
tail -1 gpurun_out/test_bnb.log
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 40 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
for mode in 0 nores 1 0 nores 1; do
  DDL_BN_BWD_EPI=$mode timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/bench_ab.log 2>&1 || exit $?
  echo "$mode $(tail -1 gpurun_out/bench_ab.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
