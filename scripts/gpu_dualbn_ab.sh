# fused downsample-block BN apply: tests (full GPU suite), then same-box ResNet-50 A/B vs the previous library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_all_gpu.log 2>&1 || { tail -30 gpurun_out/test_all_gpu.log; exit 1; }
tail -1 gpurun_out/test_all_gpu.log
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2 3; do
  for arm in 1 0; do
    DDL_DUAL_BN=$arm timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/abdual_${arm}_$i.log 2>&1 || exit $?
    echo "r50 dualbn=$arm run=$i $(val gpurun_out/abdual_${arm}_$i.log)"
  done
done
