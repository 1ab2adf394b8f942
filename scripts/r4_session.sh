#!/bin/bash
# Round-4 GPU session steps (run through gpurun on the MI355X box):
#   bash scripts/r4_session.sh STEP [STEP ...]
#   stamps      per-tile / per-k-step GEMM timeline + sampled correctness, deep retire on (d1) / off (d0)
#   gemmtests   GEMM + drain-acc + comm GPU tests
#   bertx N     N fresh-process BERT-base bench runs (30 steps): spread + GEMM plan digests
#   both        bench.py default (ResNet-50 + BERT-base)
# Each step runs under its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPES="0 16384 768 768 32 16384 768 768 0 16384 3072 768 0 16384 2304 768 32 16384 2304 768 0 16384 768 3072 32 16384 768 3072 1 16384 768 768 33 16384 768 768 1 16384 3072 768 1 16384 768 3072 0 8192 8192 8192 0 1000 1000 1000 1 4100 300 520"
while [ $# -gt 0 ]; do
  s=$1; shift
  case $s in
    stamps)
      for v in d0 d1 d2; do
        [ -x build/gemm_stamps_$v ] || continue
        timeout -k 10 150 build/gemm_stamps_$v $SHAPES > gpurun_out/stamps_$v.log 2>&1 || { tail -5 gpurun_out/stamps_$v.log; exit 1; }
        echo "== $v"; grep -E "^mode|check|k-pair|waves 0-3" gpurun_out/stamps_$v.log
      done ;;
    stampsdirect0)
      # LDS-staged epilogue (row-contiguous full-line stores, no persistent grid) vs the register epilogue
      DDL_GEMM_DIRECT=0 timeout -k 10 150 build/gemm_stamps_d1 0 16384 768 768 0 16384 3072 768 > gpurun_out/stamps_direct0.log 2>&1 \
        || { tail -5 gpurun_out/stamps_direct0.log; exit 1; }
      echo "== direct0"; grep -E "^mode|check|waves 0-3" gpurun_out/stamps_direct0.log ;;
    stampsepilds)
      # whole-row stores through LDS for plain bf16 tiles (DDL_GEMM_EPI_LDS=1) vs the register epilogue
      for v in d0 d2; do
        DDL_GEMM_EPI_LDS=1 timeout -k 10 150 build/gemm_stamps_$v 0 16384 768 768 0 16384 3072 768 0 16384 2304 768 \
          > gpurun_out/stamps_epilds_$v.log 2>&1 || { tail -5 gpurun_out/stamps_epilds_$v.log; exit 1; }
        echo "== epilds $v"; grep -E "^mode|check|waves 0-3" gpurun_out/stamps_epilds_$v.log
      done ;;
    gemmtests)
      timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_comm_gpu.py "tests/test_kernels_gpu.py::test_drain_acc" \
        -x -q --timeout 150 --timeout-method thread > gpurun_out/gemmtests.log 2>&1 || { tail -30 gpurun_out/gemmtests.log; exit 1; }
      tail -2 gpurun_out/gemmtests.log ;;
    abdr)
      # same-box BERT-base A/B: the library's retire depth vs libddl_dr2.so (DDL_DEEP_RETIRE=2), alternating
      for i in 1 2; do
        for arm in base dr2; do
          if [ $arm = dr2 ]; then export DDL_NATIVE_LIB=$PWD/databricks_distributed_deep_learning_amd/_native/ab/libddl_dr2.so; else unset DDL_NATIVE_LIB; fi
          timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/abdr_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/abdr_${arm}_$i.log; exit 1; }
          tail -1 gpurun_out/abdr_${arm}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("abdr", "'$arm'", d["value"], d.get("phases_ms"))'
        done
      done
      unset DDL_NATIVE_LIB ;;
    plans)
      # same-box BERT-base A/B of fixed GEMM plans (tune cache pre-filled from scripts/plans/*.json) and
      # the retire-depth-0 library, alternating: ARM = plan[:lib]
      for i in 1 2; do
        for arm in ${PLAN_ARMS:-bert_cur bert_bigtn bert_bigtn:dr0 bert_bigtn_b256}; do
          pl=${arm%%:*}; lib=${arm#*:}
          if [ "$lib" = dr0 ]; then export DDL_NATIVE_LIB=$PWD/databricks_distributed_deep_learning_amd/_native/ab/libddl_dr0.so; else unset DDL_NATIVE_LIB; fi
          cp scripts/plans/$pl.json gpurun_out/plan_cache.json
          DDL_GEMM_TUNE_CACHE=$PWD/gpurun_out/plan_cache.json timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 \
            > gpurun_out/plans_${arm/:/_}_$i.log 2>&1 || { tail -20 gpurun_out/plans_${arm/:/_}_$i.log; exit 1; }
          tail -1 gpurun_out/plans_${arm/:/_}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("plan", "'$arm'", d["value"], d.get("phases_ms"))'
        done
      done
      unset DDL_NATIVE_LIB ;;
    bertx)
      n=3
      if [[ ${1:-} =~ ^[0-9]+$ ]]; then n=$1; shift; fi
      for i in $(seq 1 "$n"); do
        timeout -k 10 300 python bench.py --model bert_base --steps 30 --warmup 5 > gpurun_out/bertx_$i.log 2>&1 || { tail -20 gpurun_out/bertx_$i.log; exit 1; }
        tail -1 gpurun_out/bertx_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("bert run", d["value"], d.get("gemm_plan"), d.get("phases_ms"))'
      done ;;
    arms)
      # native and stock PyTorch-ROCm arms of all four BASELINE workloads, same box, one call
      for m in resnet50 bert_base vit_b16 bert_large; do
        for arm in auto stock; do
          timeout -k 10 400 python bench.py --model $m --native $arm --steps 15 --warmup 4 > gpurun_out/arm_${m}_$arm.log 2>&1 \
            || { tail -20 gpurun_out/arm_${m}_$arm.log; exit 1; }
          tail -1 gpurun_out/arm_${m}_$arm.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print("arm", c["model"], c["native_kernels"], d["value"], d["unit"], "batch", c["per_gpu_batch"], "accum", c.get("grad_accum"), "ms", d["ms_per_step"])'
        done
      done ;;
    both)
      timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_both.log 2>&1 || { tail -20 gpurun_out/bench_both.log; exit 1; }
      tail -1 gpurun_out/bench_both.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
