# QKV bias gradient from the attention backward's column sums: tests, then same-box BERT A/B (DDL_ATTN_COLSUM)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_models_gpu.py tests/test_gemm_gpu.py tests/test_comm_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/test_attncs.log 2>&1 || { tail -30 gpurun_out/test_attncs.log; exit 1; }
tail -1 gpurun_out/test_attncs.log
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2 3; do
  for arm in 1 0; do
    DDL_ATTN_COLSUM=$arm timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/abacs_${arm}_$i.log 2>&1 || exit $?
    echo "bert attn_colsum=$arm run=$i $(val gpurun_out/abacs_${arm}_$i.log)"
  done
done
