set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fusions_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_fus.log 2>&1 || { tail -30 gpurun_out/test_fus.log; exit 1; }
tail -2 gpurun_out/test_fus.log
C="bigs 0 802816 256 64 1"
exit_after_sweep=0
C=""
for s in "200704 512 128"; do C="$C big 0 $s 1 bigs 0 $s 1"; done
timeout -k 10 120 build/gemm_sweep $C > gpurun_out/stats_sweep.log 2>&1 || exit $?
cat gpurun_out/stats_sweep.log
for e in 1 0; do
  DDL_BN_STATS_EPI=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e$e -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_e$e.log 2>&1 || exit $?
  tail -1 gpurun_out/prof_e$e.log | cut -c1-120
done
