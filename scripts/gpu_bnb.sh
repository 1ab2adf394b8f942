# BN backward reduction in the dgrad epilogue: kernel + model tests, ResNet kernel table, bench A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fusions_gpu.py tests/test_models_gpu.py tests/test_gemm_gpu.py tests/test_comm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_bnb.log 2>&1; rc=$?
tail -2 gpurun_out/test_bnb.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/test_bnb.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_r50/run_results.db --steps 5 --after sgd_k:3 --names "ResNet-50 bs256 (SGD), 1x MI355X, steady state" --top 45 > gpurun_out/kernels_r50.md
rm -rf gpurun_out/prof_r50
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 30 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
DDL_BN_BWD_EPI=0 timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_off.log 2>&1 || exit $?
tail -1 gpurun_out/bench_off.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
