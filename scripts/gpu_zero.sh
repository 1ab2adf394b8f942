set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_comm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_zero.log 2>&1; rc=$?
tail -2 gpurun_out/test_zero.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/test_zero.log | head -20; exit $rc; }
bash scripts/rehearse_world2_zero.sh > gpurun_out/rehearse_zero.log 2>&1; rc=$?; echo "rehearse rc=$rc"; grep -E "^\{|\[bench\]|Error|error" gpurun_out/rehearse_zero.log | cut -c1-300 | tail -6
