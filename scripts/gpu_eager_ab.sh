# optimizer updates during backward on a side stream: equivalence tests, then same-box A/B on both models
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_comm_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/test_eager.log 2>&1 || { tail -30 gpurun_out/test_eager.log; exit 1; }
tail -1 gpurun_out/test_eager.log
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2 3; do
  for arm in 1 0; do
    DDL_EAGER_OPTIMIZER=$arm timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/abeb_${arm}_$i.log 2>&1 || exit $?
    echo "bert eager=$arm run=$i $(val gpurun_out/abeb_${arm}_$i.log)"
  done
done
for i in 1 2; do
  for arm in 1 0; do
    DDL_EAGER_OPTIMIZER=$arm timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/aber_${arm}_$i.log 2>&1 || exit $?
    echo "r50 eager=$arm run=$i $(val gpurun_out/aber_${arm}_$i.log)"
  done
done
