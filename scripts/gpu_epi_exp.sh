set -o pipefail
mkdir -p gpurun_out
C="big 0 16384 3072 256 1 big 0 16384 3072 768 1 big 0 16384 3072 3072 1 big 0 16384 768 768 1 big 0 16384 2304 768 1 big 0 8192 8192 8192 1 big 1 16384 768 3072 1"
rm -f gpurun_out/epi_exp.log
for e in 0 3 0 3; do
  echo "== epi$e" >> gpurun_out/epi_exp.log
  timeout -k 10 120 build/gemm_sweep_epi$e $C >> gpurun_out/epi_exp.log 2>&1 || exit $?
done
