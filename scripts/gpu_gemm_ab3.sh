# kernel-level A/B (standalone GEMM times, no occupant) of the current library against
# scripts/build_ab.sh's "base" build, then the full bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_fusions_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1; rc=$?; tail -2 gpurun_out/t_gemm.log; [ $rc -eq 0 ] || exit $rc
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
    print(f"{k:26s} base {min(v['base']):.4f}  cur {min(v['cur']):.4f}  ratio {min(v['base'])/min(v['cur']):.3f}")
PY
bash scripts/gpu_lib_ab.sh base 2
