# LayerNorm backward grid sweep (rows per block x block cap), BERT-base shape; kernel time from rocprofv3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "16 1024" "32 1024" "8 2048" "32 512" "64 256" "16 1024"; do
  set -- $cfg
  rm -rf gpurun_out/ln_prof
  DDL_LN_BWD_ROWS=$1 DDL_LN_BWD_MAXBLK=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ln_prof -o run -- python3 scripts/debug/ln_bwd_bench.py > gpurun_out/ln_prof.log 2>&1 || exit 1
  echo "$1 $2 $(python3 scripts/prof_summary.py gpurun_out/ln_prof/run_results.db --steps 1 --top 8 | grep -E 'ln_bwd_k|colsum_partials_k|collapse' | awk -F'|' '{printf "%s %s us; ", $2, $5}')"
done
rm -rf gpurun_out/ln_prof
