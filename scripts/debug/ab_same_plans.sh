# Same-box A/B of a kernel-source change that alters the GEMM source hash: the tree's library vs
# ab/libddl_old.so (scripts/build_ab.sh HEAD old <changed files>), both on ab/gemm_plans_new.json (the
# committed plans re-keyed to the tree's GEMM source hash, so both arms run the same kernel choices):
#   bash scripts/debug/ab_same_plans.sh [MICROBENCH.py]   -> the microbenchmark in each arm, then bench.py x3
set -o pipefail
A=$PWD/databricks_distributed_deep_learning_amd/_native/ab
export DDL_GEMM_PLAN_TABLE=$A/gemm_plans_new.json
if [ -n "$1" ]; then
  for arm in new old; do
    if [ $arm = old ]; then export DDL_NATIVE_LIB=$A/libddl_old.so; else unset DDL_NATIVE_LIB; fi
    timeout -k 10 200 python "$1" > gpurun_out/abm_$arm.log 2>&1 || { tail -20 gpurun_out/abm_$arm.log; exit 1; }
    echo "[$arm]"; grep -v amdgpu.ids gpurun_out/abm_$arm.log
  done
fi
for i in 1 2 3; do
  for arm in new old; do
    if [ $arm = old ]; then export DDL_NATIVE_LIB=$A/libddl_old.so; else unset DDL_NATIVE_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/abr_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/abr_${arm}_$i.log; exit 1; }
    echo "$arm $i $(grep '^{' gpurun_out/abr_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["bert_base_samples_per_sec"], d["plan_source"]["source"], d["plan_source"]["misses"])')"
  done
done
