# dual-BN downsample apply + fused stem: full GPU suite, then same-box ResNet-50 A/B of both toggles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_all_gpu.log 2>&1 || { tail -30 gpurun_out/test_all_gpu.log; exit 1; }
tail -1 gpurun_out/test_all_gpu.log
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2 3; do
  for arm in "1 1" "0 1" "1 0"; do
    set -- $arm
    DDL_DUAL_BN=$1 DDL_FUSED_STEM=$2 timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/abf_$1_$2_$i.log 2>&1 || exit $?
    echo "r50 dualbn=$1 stem=$2 run=$i $(val gpurun_out/abf_$1_$2_$i.log)"
  done
done
