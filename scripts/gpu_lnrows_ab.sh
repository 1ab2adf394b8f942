# LayerNorm backward rows per block after the pipelining (DDL_LN_BWD_ROWS): same-box BERT A/B
set -o pipefail
mkdir -p gpurun_out
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2; do
  for arm in 32 16 64; do
    DDL_LN_BWD_ROWS=$arm timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/ablnr_${arm}_$i.log 2>&1 || exit $?
    echo "bert ln_rows=$arm run=$i $(val gpurun_out/ablnr_${arm}_$i.log)"
  done
done
