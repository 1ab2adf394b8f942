set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_comm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_check.log 2>&1 || { tail -30 gpurun_out/test_check.log; exit 1; }
tail -1 gpurun_out/test_check.log
timeout -k 10 120 build/gemm_sweep big 2 2304 768 16384 8 big 2 2304 768 16384 9 big 2 3072 768 16384 8 big 2 768 768 16384 8 big 2 768 3072 16384 8 > gpurun_out/tn_sweep.log 2>&1 && cat gpurun_out/tn_sweep.log
bash scripts/rehearse_world2.sh > gpurun_out/rehearse.log 2>&1; rc=$?; echo "rehearse rc=$rc"; tail -3 gpurun_out/rehearse.log | cut -c1-300
