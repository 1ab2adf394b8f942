# GEMM numerics + microbench + full bench: HEAD gemm_big ("base") vs the current build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_fusions_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1; rc=$?; tail -1 gpurun_out/t_gemm.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_gemm.log | head; exit $rc; }
DDL_GEMM_BEHIND=7 timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_gemm7.log 2>&1; rc=$?; tail -1 gpurun_out/t_gemm7.log; [ $rc -eq 0 ] || exit $rc
B=$PWD/databricks_distributed_deep_learning_amd/_native/ab/libddl_base.so
for i in 1 2; do
DDL_NATIVE_LIB=$B timeout -k 10 200 python benchmarks/comm_overlap.py --occupy 0 > gpurun_out/ov_base_$i.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/comm_overlap.py --occupy 0 > gpurun_out/ov_cur_$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/ov_*_?.log")):
    arm = f.split("_")[2]
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); rows.setdefault(d["shape"], {}).setdefault(arm, []).append(d["alone_ms"])
for k, v in rows.items():
    print(f"{k:26s} " + "  ".join(f"{a} {min(v[a]):.4f}" for a in ("base", "cur", "b7") if a in v))
PY
for i in 1 2; do
  for arm in base cur; do
    case $arm in base) export DDL_NATIVE_LIB=$B; unset DDL_GEMM_BEHIND;; cur) unset DDL_NATIVE_LIB DDL_GEMM_BEHIND;; b7) unset DDL_NATIVE_LIB; export DDL_GEMM_BEHIND=7;; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/abb_${arm}_$i.log 2>&1 || exit $?
    echo "$arm run=$i $(tail -1 gpurun_out/abb_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["bert_base_samples_per_sec"])')"
  done
done
