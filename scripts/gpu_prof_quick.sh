# kernel tables (rocprofv3 --kernel-trace --stats) + per-GEMM traces of both models
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python3 bench.py --model bert_base --steps 5 --warmup 3 > gpurun_out/prof_bert.log 2>&1 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_r50/run_results.db --steps 5 --after sgd_k:3 --names "ResNet-50 bs256 (SGD), 1x MI355X, steady state" --top 60 > gpurun_out/kernels_r50.md
python3 scripts/prof_summary.py gpurun_out/prof_bert/run_results.db --steps 5 --after adamw_k:3 --names "BERT-base bs128 s128 (AdamW), 1x MI355X, steady state" --top 45 > gpurun_out/kernels_bert.md
rm -rf gpurun_out/prof_r50 gpurun_out/prof_bert
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 50 > gpurun_out/gemm_trace_r50.md 2> gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
timeout -k 10 300 python scripts/debug/gemm_trace.py bert_base --top 30 > gpurun_out/gemm_trace_bert.md 2> gpurun_out/gemm_trace_bert.err || { tail -20 gpurun_out/gemm_trace_bert.err; exit 1; }
