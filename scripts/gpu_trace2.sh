# per-GEMM traces of one training step (ResNet-50, BERT-base)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/debug/gemm_trace.py resnet50 --top 60 > gpurun_out/gemm_trace_r50.md 2>gpurun_out/gemm_trace_r50.err || { tail -20 gpurun_out/gemm_trace_r50.err; exit 1; }
timeout -k 10 300 python scripts/debug/gemm_trace.py bert_base --top 30 > gpurun_out/gemm_trace_bert.md 2>gpurun_out/gemm_trace_bert.err || { tail -20 gpurun_out/gemm_trace_bert.err; exit 1; }
head -3 gpurun_out/gemm_trace_r50.md
