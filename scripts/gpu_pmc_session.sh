set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 build/gemm_sweep > gpurun_out/gemm_sweep.log 2>&1 && \
bash scripts/pmc_profile.sh gpurun_out/pmc_gemm -- build/gemm_sweep big 0 16384 3072 768 1 big 0 8192 8192 8192 1 big 2 2304 768 16384 4 small 0 16384 3072 768 1 && \
bash scripts/pmc_profile.sh gpurun_out/pmc_r50 -- python3 bench.py --model resnet50 --steps 2 --warmup 1 && \
bash scripts/pmc_profile.sh gpurun_out/pmc_bert -- python3 bench.py --model bert_base --steps 2 --warmup 1
