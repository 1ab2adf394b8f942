set -o pipefail
mkdir -p gpurun_out
C="big 0 16384 3072 256 1 big 0 16384 3072 768 1 big 0 16384 3072 3072 1 big 0 16384 768 768 1 big 0 16384 2304 768 1 big 0 8192 8192 8192 1 big 1 16384 768 3072 1 big 1 16384 3072 768 1 big 2 2304 768 16384 8 big 2 3072 768 16384 4"
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_gemm.log 2>&1 || { tail -30 gpurun_out/test_gemm.log; exit 1; }
tail -2 gpurun_out/test_gemm.log
rm -f gpurun_out/direct_ab.log
for d in 1 0 1; do
  echo "== DDL_GEMM_DIRECT=$d" >> gpurun_out/direct_ab.log
  DDL_GEMM_DIRECT=$d timeout -k 10 120 build/gemm_sweep $C >> gpurun_out/direct_ab.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
