# persistent prefetching short attention forward + no-scratch staging: attention / model tests, BERT A/B vs HEAD lib
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_models_gpu.py tests/test_race_screen_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/test_attnp.log 2>&1 || { tail -30 gpurun_out/test_attnp.log; exit 1; }
tail -1 gpurun_out/test_attnp.log
bash scripts/gpu_ab_bert.sh attnold
