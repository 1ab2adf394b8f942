# same-box A/B of a library variant on the BERT-base half of the bench (3 alternating runs)
set -o pipefail
mkdir -p gpurun_out
V=$PWD/databricks_distributed_deep_learning_amd/_native/ab/libddl_$1.so
for i in 1 2 3; do
  for arm in cur $1; do
    if [ $arm = cur ]; then unset DDL_NATIVE_LIB; else export DDL_NATIVE_LIB=$V; fi
    timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/abbert_${arm}_$i.log 2>&1 || exit $?
    echo "$arm run=$i $(tail -1 gpurun_out/abbert_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
