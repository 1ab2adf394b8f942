set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for e in 1 0; do
  DDL_BN_STATS_EPI=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e$e -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_e$e.log 2>&1 || exit $?
  tail -1 gpurun_out/prof_e$e.log | cut -c1-120
done
