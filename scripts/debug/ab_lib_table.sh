set -o pipefail
A=$PWD/databricks_distributed_deep_learning_amd/_native/ab
for i in 1 2 3; do
  for arm in new old; do
    if [ $arm = old ]; then export DDL_NATIVE_LIB=$A/libddl_old.so DDL_GEMM_PLAN_TABLE=$A/gemm_plans_old.json; else unset DDL_NATIVE_LIB DDL_GEMM_PLAN_TABLE; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/abl_${arm}_$i.log 2>&1 || exit 1
    echo "$arm $i $(grep '^{' gpurun_out/abl_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["bert_base_samples_per_sec"], d["plan_source"]["source"], d["plan_source"]["misses"])')"
  done
done
