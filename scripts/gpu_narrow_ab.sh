# 128x64 tiles as a tuner candidate for statistics / BN-backward epilogues: gemm + fusion tests, same-box A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fusions_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_narrow.log 2>&1 || { tail -30 gpurun_out/test_narrow.log; exit 1; }
tail -1 gpurun_out/test_narrow.log
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2 3; do
  for arm in 1 0; do
    DDL_TUNE_NARROW_STATS=$arm timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/abnar_${arm}_$i.log 2>&1 || exit $?
    echo "r50 narrow_stats=$arm run=$i $(val gpurun_out/abnar_${arm}_$i.log)"
  done
done
