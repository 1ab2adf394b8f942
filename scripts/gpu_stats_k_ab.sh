# In-run A/B: forward BN statistics epilogue threshold (DDL_BN_STATS_MIN_K) after the DPP stats reduction.
set -o pipefail
mkdir -p gpurun_out
for k in 2048 0 576 2048 0 576; do
  DDL_BN_STATS_MIN_K=$k timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/bench_ab.log 2>&1 || exit $?
  echo "$k $(tail -1 gpurun_out/bench_ab.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
