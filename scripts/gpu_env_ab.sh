# same-box A/B of an environment setting on one half of the bench (3 alternating runs):
#   bash scripts/gpu_env_ab.sh <model> "<env for arm A>" "<env for arm B>"
set -o pipefail
mkdir -p gpurun_out
m=$1; A=$2; B=$3
for i in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 > gpurun_out/envab_${arm}_$i.log 2>&1 || exit $?
    echo "$arm [$E] run=$i $(tail -1 gpurun_out/envab_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
