# Same-box A/B of the split-K reduce: the tree's library vs ab/libddl_old.so (scripts/build_ab.sh HEAD old
# csrc/kernels/gemm_duo.hip), both on ab/gemm_plans_new.json (the committed plans re-keyed to the tree's GEMM
# source hash, so both arms run the same kernel choices): isolated TN GEMMs, then bench.py alternating.
set -o pipefail
A=$PWD/databricks_distributed_deep_learning_amd/_native/ab
export DDL_GEMM_PLAN_TABLE=$A/gemm_plans_new.json
for arm in new old; do
  if [ $arm = old ]; then export DDL_NATIVE_LIB=$A/libddl_old.so; else unset DDL_NATIVE_LIB; fi
  timeout -k 10 200 python scripts/debug/duo_tn_reduce_bench.py > gpurun_out/redb_$arm.log 2>&1 || { tail -20 gpurun_out/redb_$arm.log; exit 1; }
  cat gpurun_out/redb_$arm.log | grep TN
done
for i in 1 2 3; do
  for arm in new old; do
    if [ $arm = old ]; then export DDL_NATIVE_LIB=$A/libddl_old.so; else unset DDL_NATIVE_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/abr_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/abr_${arm}_$i.log; exit 1; }
    echo "$arm $i $(grep '^{' gpurun_out/abr_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["bert_base_samples_per_sec"], d["plan_source"]["source"], d["plan_source"]["misses"])')"
  done
done
