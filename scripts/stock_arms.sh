set -o pipefail
mkdir -p gpurun_out/stock
for m in resnet50 bert_base vit_b16; do
  for arm in auto stock; do
    timeout -k 10 300 python bench.py --model $m --native $arm --steps 15 --warmup 4 > gpurun_out/stock/${m}_${arm}.log 2>&1 || exit 1
    echo "arm $m $arm $(tail -1 gpurun_out/stock/${m}_${arm}.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], "batch", d["config"]["per_gpu_batch"], "accum", d["config"]["grad_accum"], "ms", d["ms_per_step"])')"
  done
done
for arm in auto stock; do
  timeout -k 10 400 python bench.py --model bert_large --batch 472 --native $arm --steps 3 --warmup 1 > gpurun_out/stock/bert_large_${arm}.log 2>&1 || exit 1
  echo "arm bert_large $arm $(tail -1 gpurun_out/stock/bert_large_${arm}.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], "batch", d["config"]["per_gpu_batch"], "accum", d["config"]["grad_accum"], "ms", d["ms_per_step"])')"
done
