# ResNet-50: selected GPU tests, steady-state kernel table, bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_gemm_gpu.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/test_r50p.log 2>&1; rc=$?
tail -1 gpurun_out/test_r50p.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/test_r50p.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_r50/run_results.db --steps 5 --after sgd_k:3 --names "ResNet-50 bs256 (SGD), 1x MI355X, steady state" --top 45 > gpurun_out/kernels_r50.md
rm -rf gpurun_out/prof_r50
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
