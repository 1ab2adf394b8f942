# skinny residual + BN-backward epilogue: tests, then same-box A/B (DDL_SKINNY_RESBNB)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_skinny_gemm_gpu.py tests/test_fusions_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_resbnb.log 2>&1 || { tail -30 gpurun_out/test_resbnb.log; exit 1; }
tail -1 gpurun_out/test_resbnb.log
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2 3; do
  for arm in 0 1; do
    DDL_SKINNY_RESBNB=$arm timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/abrb_${arm}_$i.log 2>&1 || exit $?
    echo "r50 resbnb=$arm run=$i $(val gpurun_out/abrb_${arm}_$i.log)"
  done
done
timeout -k 10 300 python scripts/debug/tn_wgrad_vs_blaslt.py > gpurun_out/tn_wgrad_vs_blaslt.log 2>&1 || { tail -20 gpurun_out/tn_wgrad_vs_blaslt.log; exit 1; }
cat gpurun_out/tn_wgrad_vs_blaslt.log
