# Slice size of the merged BatchNorm / LayerNorm finalize (DDL_FIN_RPS) against the BN finalize
# microbenchmark (every ResNet-50 shape) and the BERT-base LayerNorm backward (which includes its
# column-sum finalize)
set -o pipefail
for r in 128 64 32; do
  echo "== DDL_FIN_RPS=$r"
  DDL_FIN_RPS=$r timeout -k 10 120 python scripts/debug/fin_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
  DDL_FIN_RPS=$r timeout -k 10 120 python scripts/debug/ln_bwd_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
