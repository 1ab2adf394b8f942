# Round-end evidence: full GPU suite, smoke, bench line, BERT-base kernel table (attention changed last)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/test_all_gpu.log 2>&1 || { tail -30 gpurun_out/test_all_gpu.log; exit 1; }
tail -1 gpurun_out/test_all_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || exit $?
tail -1 gpurun_out/bench_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python3 bench.py --model bert_base --steps 5 --warmup 3 > gpurun_out/prof_bert.log 2>&1 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_bert/run_results.db --steps 5 --after adamw_k:3 --names "BERT-base bs128 s128 (AdamW), 1x MI355X, steady state" --top 40 > gpurun_out/kernels_bert.md; rm -rf gpurun_out/prof_bert
head -12 gpurun_out/kernels_bert.md
