#!/bin/bash
# same-box comparison of several environment settings on one half of the bench (2 rounds):
#   bash scripts/gpu_env_ab3.sh <model> "<env 1>" "<env 2>" ["<env 3>" ...]
set -o pipefail
mkdir -p gpurun_out
m=$1; shift
for i in 1 2; do
  k=0
  for E in "$@"; do
    k=$((k + 1))
    env $E timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 > gpurun_out/envab3_${k}_$i.log 2>&1 || exit $?
    echo "[$E] run=$i $(tail -1 gpurun_out/envab3_${k}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
