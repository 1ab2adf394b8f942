# In-model kernel tables (BERT-base) for the split-K reduce A/B: tree library vs ab/libddl_old.so, both on
# ab/gemm_plans_new.json (see ab_same_plans.sh)
set -o pipefail
A=$PWD/databricks_distributed_deep_learning_amd/_native/ab
export DDL_GEMM_PLAN_TABLE=$A/gemm_plans_new.json
for arm in new old; do
  if [ $arm = old ]; then export DDL_NATIVE_LIB=$A/libddl_old.so; else unset DDL_NATIVE_LIB; fi
  timeout -k 10 200 python scripts/debug/duo_tn_reduce_bench.py > gpurun_out/redb_$arm.log 2>&1 || { tail -20 gpurun_out/redb_$arm.log; exit 1; }
  grep TN gpurun_out/redb_$arm.log
  bash scripts/gpu.sh "prof bert_base" > /dev/null 2>&1 || exit 1
  cp gpurun_out/kernels_bert_base.md gpurun_out/kb_red_$arm.md
  grep -E "GPU busy|duo_reduce|gemm_duo_k<1, 1" gpurun_out/kb_red_$arm.md
done
