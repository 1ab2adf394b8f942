# same-box A/B: DDL_BN_BWD_EPI (nores vs 1: BN-backward epilogue also on residual-adding dgrads,
# residual gradient handed on as the dgrad output itself), DDL_WDG_BATCH (per-step batched
# conv dgrad weight layouts), DDL_LN_BIAS_SINK (LayerNorm backward writes the Linear bias grad)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fusions_gpu.py tests/test_models_gpu.py tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/test_bnres.log 2>&1 || { tail -30 gpurun_out/test_bnres.log; exit 1; }
tail -1 gpurun_out/test_bnres.log
val() { tail -1 $1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for i in 1 2; do
  for arm in "nores 0" "nores 1" "1 1"; do
    set -- $arm
    DDL_BN_BWD_EPI=$1 DDL_WDG_BATCH=$2 timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 5 > gpurun_out/abres_$1_$2_$i.log 2>&1 || exit $?
    echo "r50 epi=$1 batch=$2 run=$i $(val gpurun_out/abres_$1_$2_$i.log)"
  done
  for sk in 0 1; do
    DDL_LN_BIAS_SINK=$sk timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/absink_${sk}_$i.log 2>&1 || exit $?
    echo "bert sink=$sk run=$i $(val gpurun_out/absink_${sk}_$i.log)"
  done
done
