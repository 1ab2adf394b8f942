# BN partial-row collapse threshold (DDL_BN_COLLAPSE_MIN): same-box A/B on both models
set -o pipefail
mkdir -p gpurun_out
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2; do
  for arm in 0 1024 4096; do
    DDL_BN_COLLAPSE_MIN=$arm timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/abcol_${arm}_$i.log 2>&1 || exit $?
    echo "r50 collapse_min=$arm run=$i $(val gpurun_out/abcol_${arm}_$i.log)"
  done
done
for i in 1 2; do
  for arm in 0 1024; do
    DDL_BN_COLLAPSE_MIN=$arm timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/abcolb_${arm}_$i.log 2>&1 || exit $?
    echo "bert collapse_min=$arm run=$i $(val gpurun_out/abcolb_${arm}_$i.log)"
  done
done
