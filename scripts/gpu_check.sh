set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_all.log 2>&1; rc=$?
tail -3 gpurun_out/test_all.log
[ $rc -eq 0 ] || { grep -E "Error|error|FAILED|assert" gpurun_out/test_all.log | head -20; exit $rc; }
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
