# A/B of two builds of the kernel library on the full bench, alternating arms:
#   bash scripts/gpu_lib_ab.sh <variant-name> [reps]   (variant built by scripts/build_ab.sh)
set -o pipefail
mkdir -p gpurun_out
v=$1; reps=${2:-2}
lib=databricks_distributed_deep_learning_amd/_native/ab/libddl_$v.so
for i in $(seq 1 $reps); do
  for arm in cur $v; do
    if [ $arm = cur ]; then unset DDL_NATIVE_LIB; else export DDL_NATIVE_LIB=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_${arm}_$i.log 2>&1 || exit $?
    echo "$arm run=$i $(tail -1 gpurun_out/ab_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["bert_base_samples_per_sec"])')"
  done
done
