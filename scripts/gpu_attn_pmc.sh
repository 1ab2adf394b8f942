# hardware counters for the attention kernels (BERT-base shape only)
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_attn
bash scripts/pmc_profile.sh gpurun_out/pmc_attn -- python3 benchmarks/attention_bench.py --shapes bert_base || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_attn --match attn > gpurun_out/pmc_attn.md
cat gpurun_out/pmc_attn.md
