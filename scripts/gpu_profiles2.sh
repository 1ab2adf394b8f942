# Evidence refresh without the standalone GEMM binary: bench line, rocprofv3 kernel tables and PMC
# passes for both models; every raw trace is summarised and deleted right away (gpurun_out <= 64 MiB)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DDL_GEMM_TUNE_CACHE=$PWD/gpurun_out/tune_cache.json
rm -f "$DDL_GEMM_TUNE_CACHE"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || exit $?
tail -1 gpurun_out/bench_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_r50/run_results.db --steps 5 --after sgd_k:3 --names "ResNet-50 bs256 (SGD), 1x MI355X, steady state" --top 45 > gpurun_out/kernels_r50.md; rm -rf gpurun_out/prof_r50
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python3 bench.py --model bert_base --steps 5 --warmup 3 > gpurun_out/prof_bert.log 2>&1 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_bert/run_results.db --steps 5 --after adamw_k:3 --names "BERT-base bs128 s128 (AdamW), 1x MI355X, steady state" --top 40 > gpurun_out/kernels_bert.md; rm -rf gpurun_out/prof_bert
rm -rf gpurun_out/pmc_r50 gpurun_out/pmc_bert
bash scripts/pmc_profile.sh gpurun_out/pmc_r50 -- python3 bench.py --model resnet50 --steps 2 --warmup 1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_r50 --top 30 --title "ResNet-50 bs256 training step (1 warm-up + 2 steps, tuned kernel choices from cache)" > gpurun_out/pmc_r50.md; rm -rf gpurun_out/pmc_r50
bash scripts/pmc_profile.sh gpurun_out/pmc_bert -- python3 bench.py --model bert_base --steps 2 --warmup 1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_bert --top 30 --title "BERT-base bs128 s128 training step (1 warm-up + 2 steps, tuned kernel choices from cache)" > gpurun_out/pmc_bert.md; rm -rf gpurun_out/pmc_bert
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 50 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
timeout -k 10 300 python scripts/debug/gemm_trace.py bert_base --top 30 > gpurun_out/gemm_trace_bert.md 2> gpurun_out/gemm_trace_bert.err || { tail -20 gpurun_out/gemm_trace_bert.err; exit 1; }
