# Refresh the committed evidence: bench line, rocprofv3 kernel tables (ResNet-50 and
# BERT-base steady state), PMC counter passes (tuner choices loaded from a cache so
# no candidate-timing dispatches pollute the counters), standalone GEMM sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DDL_GEMM_TUNE_CACHE=$PWD/gpurun_out/tune_cache.json
rm -f "$DDL_GEMM_TUNE_CACHE"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || exit $?
tail -1 gpurun_out/bench_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python3 bench.py --model bert_base --steps 5 --warmup 3 > gpurun_out/prof_bert.log 2>&1 || exit $?
rm -rf gpurun_out/pmc_r50 gpurun_out/pmc_bert gpurun_out/pmc_gemm
bash scripts/pmc_profile.sh gpurun_out/pmc_r50 -- python3 bench.py --model resnet50 --steps 2 --warmup 1 || exit $?
bash scripts/pmc_profile.sh gpurun_out/pmc_bert -- python3 bench.py --model bert_base --steps 2 --warmup 1 || exit $?
bash scripts/pmc_profile.sh gpurun_out/pmc_gemm -- build/gemm_sweep big 0 16384 3072 768 1 big 0 8192 8192 8192 1 big 2 2304 768 16384 8 || exit $?
timeout -k 10 240 build/gemm_sweep > gpurun_out/gemm_sweep.log 2>&1
# summarise on the box (raw counter CSVs are too large to ship back)
python3 scripts/prof_summary.py gpurun_out/prof_r50/run_results.db --steps 5 --after sgd_k:3 --names "ResNet-50 bs256 (SGD), 1x MI355X, steady state" --top 40 > gpurun_out/kernels_r50.md
python3 scripts/prof_summary.py gpurun_out/prof_bert/run_results.db --steps 5 --after adamw_k:3 --names "BERT-base bs128 s128 (AdamW), 1x MI355X, steady state" --top 40 > gpurun_out/kernels_bert.md
python3 scripts/pmc_summary.py gpurun_out/pmc_r50 --top 30 --title "ResNet-50 bs256 training step (1 warm-up + 2 steps, tuned kernel choices from cache)" > gpurun_out/pmc_r50.md
python3 scripts/pmc_summary.py gpurun_out/pmc_bert --top 30 --title "BERT-base bs128 s128 training step (1 warm-up + 2 steps, tuned kernel choices from cache)" > gpurun_out/pmc_bert.md
python3 scripts/pmc_summary.py gpurun_out/pmc_gemm --top 10 --title "Standalone GEMMs: NT 16384x3072x768 / 8192^3, TN 2304x768x16384 split 8" > gpurun_out/pmc_gemm.md
rm -rf gpurun_out/pmc_r50 gpurun_out/pmc_bert gpurun_out/pmc_gemm gpurun_out/prof_r50 gpurun_out/prof_bert
