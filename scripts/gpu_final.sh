# Round-end rehearsal: full GPU suite, smoke(), bench (ResNet-50 + BERT-base), per-GEMM trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_all_gpu.log 2>&1 || { tail -30 gpurun_out/test_all_gpu.log; exit 1; }
tail -1 gpurun_out/test_all_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 45 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
echo done
