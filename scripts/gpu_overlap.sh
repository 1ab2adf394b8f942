set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_fusions_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1; rc=$?; tail -2 gpurun_out/t_gemm.log; [ $rc -eq 0 ] || exit $rc
DDL_GEMM_DYNAMIC=1 timeout -k 10 200 python benchmarks/comm_overlap.py > gpurun_out/overlap_dyn.log 2>&1 || exit $?
bash scripts/gpu_lib_ab.sh base 2
