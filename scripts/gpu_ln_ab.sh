# pipelined LayerNorm backward: LN tests, then same-box BERT A/B against the previous kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "layernorm or layer_norm or bert or vit" > gpurun_out/test_ln.log 2>&1 || { tail -30 gpurun_out/test_ln.log; exit 1; }
tail -1 gpurun_out/test_ln.log
bash scripts/gpu_ab_bert.sh lnold
