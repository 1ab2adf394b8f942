#!/bin/bash
# One parametrised GPU harness (run on the MI355X box through gpurun):
#
#   bash scripts/gpu.sh STEP [STEP ...]       e.g.  bash scripts/gpu.sh tests smoke bench "prof resnet50"
#
# Steps (each under its own time limit; the script stops at the first failing step):
#   tests [FILES]         GPU test suite (default all of tests/) -> gpurun_out/test_gpu.log
#   smoke                 __graft_entry__.smoke()             -> gpurun_out/smoke.log
#   bench [args]          bench.py (default 20 steps, 5 warm-up) -> gpurun_out/bench.log
#   stock [args]          bench.py --native stock (plain PyTorch-ROCm + torch DDP arm)
#   ab LIB MODEL [RUNS]   same-box A/B of libddl_LIB.so (scripts/build_ab.sh) vs the tree's library,
#                         alternating RUNS times (default 3) on MODEL (resnet50 | bert_base | vit_b16 | ...)
#   abenv VAR=VAL MODEL [RUNS]  same-box A/B of an environment toggle (unset vs VAR=VAL), alternating
#   prof MODEL            rocprofv3 kernel table (steady state) -> gpurun_out/kernels_MODEL.md
#   pmc MODEL             3 PMC passes summarised             -> gpurun_out/pmc_MODEL.md
#   presets               every BASELINE preset through the train() CLI
#   rehearse2             2 ranks on this one GPU over gloo through bench.py's own launcher
#   tuneplans             tune every benchmark / preset GEMM signature with the plan table off
#                         -> gpurun_out/plans/cache.json (scripts/make_plan_table.py turns it into
#                         ops/gemm_plans.json)
#   script FILE [args]    any python script under a 300 s limit (debug / microbenchmarks)
#
# MODEL for prof/pmc: resnet50 | bert_base (bench.py) or vit_b16 | bert_large_lamb (train CLI).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TRAIN="python3 -m databricks_distributed_deep_learning_amd.training.loop"

run_model() {   # run_model MODEL STEPS WARMUP -> command words for one profiled run
  case $1 in
    resnet50|bert_base) echo "python3 bench.py --model $1 --steps $2 --warmup $3" ;;
    vit_b16) echo "$TRAIN --preset vit_b16 --steps $2 --warmup_steps $3 --log_every 0" ;;
    bert_large_lamb) echo "$TRAIN --preset bert_large_lamb --batch_size 32 --steps $2 --warmup_steps $3 --log_every 0" ;;
    *) echo "unknown model $1" >&2; return 1 ;;
  esac
}
ab_value() {    # ab_value LOG -> the throughput of a bench.py (value) or train CLI (samples_per_sec) run
  tail -1 "$1" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d.get("value", d.get("samples_per_sec")), d.get("phases_ms") or "")'
}
opt_kernel() {  # the optimizer kernel that ends each step (steady-state cut for prof_summary)
  case $1 in resnet50) echo sgd_k ;; bert_large_lamb) echo lamb_phase2 ;; *) echo adamw_k ;; esac
}

step() {
  local name=$1; shift
  echo "=== [$name] $*" >&2
  case $name in
    tests)
      # args: test files / node ids (default: the whole tests/ directory)
      timeout -k 10 700 python -u -m pytest "${@:-tests}" -m gpu -x -q --timeout 180 --timeout-method thread \
        > gpurun_out/test_gpu.log 2>&1 || { tail -40 gpurun_out/test_gpu.log; return 1; }
      tail -1 gpurun_out/test_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { tail -20 gpurun_out/smoke.log; return 1; }
      tail -1 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/bench.log 2>&1 \
        || { tail -20 gpurun_out/bench.log; return 1; }
      grep '^\[bench\]' gpurun_out/bench.log | cut -c1-400; tail -1 gpurun_out/bench.log ;;
    stock)
      timeout -k 10 400 python bench.py --native stock --steps 20 --warmup 5 "$@" > gpurun_out/stock.log 2>&1 \
        || { tail -20 gpurun_out/stock.log; return 1; }
      tail -1 gpurun_out/stock.log ;;
    ab)
      local lib=$1 model=$2 runs=${3:-3}
      local v=$PWD/databricks_distributed_deep_learning_amd/_native/ab/libddl_$lib.so
      for i in $(seq 1 "$runs"); do
        for arm in cur "$lib"; do
          if [ "$arm" = cur ]; then unset DDL_NATIVE_LIB; else export DDL_NATIVE_LIB=$v; fi
          # shellcheck disable=SC2046
          timeout -k 10 300 $(run_model "$model" 30 5) > "gpurun_out/ab_${arm}_$i.log" 2>&1 \
            || { tail -20 "gpurun_out/ab_${arm}_$i.log"; return 1; }
          echo "$arm run=$i $(ab_value "gpurun_out/ab_${arm}_$i.log")"
        done
      done
      unset DDL_NATIVE_LIB ;;
    abenv)
      local kv=$1 model=$2 runs=${3:-3}
      for i in $(seq 1 "$runs"); do
        for arm in base env; do
          if [ "$arm" = base ]; then
            # shellcheck disable=SC2046
            timeout -k 10 300 $(run_model "$model" 30 5) > "gpurun_out/abenv_${arm}_$i.log" 2>&1 \
              || { tail -20 "gpurun_out/abenv_${arm}_$i.log"; return 1; }
          else
            # shellcheck disable=SC2046
            env "$kv" timeout -k 10 300 $(run_model "$model" 30 5) > "gpurun_out/abenv_${arm}_$i.log" 2>&1 \
              || { tail -20 "gpurun_out/abenv_${arm}_$i.log"; return 1; }
          fi
          echo "$arm($kv) $model run=$i $(ab_value "gpurun_out/abenv_${arm}_$i.log")"
        done
      done ;;
    prof)
      local m=$1 cmd
      cmd=$(run_model "$m" 5 3) || return 1
      rm -rf "gpurun_out/prof_$m"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$m" -o run -- $cmd \
        > "gpurun_out/prof_$m.log" 2>&1 || { tail -20 "gpurun_out/prof_$m.log"; return 1; }
      python3 scripts/prof_summary.py "gpurun_out/prof_$m/run_results.db" --steps 5 --after "$(opt_kernel "$m"):3" \
        --names "$m steady state, 1x MI355X" --top 45 > "gpurun_out/kernels_$m.md"
      rm -rf "gpurun_out/prof_$m"
      head -14 "gpurun_out/kernels_$m.md" ;;
    pmc)
      # 3 steady-state steps after 2 warm-up steps; the summary counts only dispatches after the
      # warm-up's last optimizer kernel (pmc_summary.py --after)
      local m=$1 cmd
      cmd=$(run_model "$m" 3 2) || return 1
      rm -rf "gpurun_out/pmc_$m"
      # tune once into a cache first: the counted runs load the GEMM kernel choices instead of
      # timing every candidate (whose dispatches would otherwise fill the table)
      export DDL_GEMM_TUNE_CACHE=$PWD/gpurun_out/tune_$m.json
      rm -f "$DDL_GEMM_TUNE_CACHE"
      timeout -k 10 300 $cmd > "gpurun_out/pmc_${m}_tune.log" 2>&1 || { tail -20 "gpurun_out/pmc_${m}_tune.log"; return 1; }
      bash scripts/pmc_profile.sh "gpurun_out/pmc_$m" -- $cmd || return 1
      unset DDL_GEMM_TUNE_CACHE
      python3 scripts/pmc_summary.py "gpurun_out/pmc_$m" --top 30 --after "$(opt_kernel "$m"):2" \
        --title "$m training step, steady state (3 steps counted after 2 warm-up steps)" > "gpurun_out/pmc_$m.md"
      rm -rf "gpurun_out/pmc_$m"
      head -14 "gpurun_out/pmc_$m.md" ;;
    presets)
      for spec in "resnet18_gloo:--backend=nccl --steps=3 --warmup_steps=1" "resnet50_ddp:--steps=3 --warmup_steps=1" \
                  "bert_base_ddp:--steps=3 --warmup_steps=1" "vit_b16:--steps=10 --warmup_steps=3" \
                  "bert_large_lamb:--steps=2 --warmup_steps=1"; do
        local pn="${spec%%:*}" pa="${spec#*:}"
        timeout -k 10 400 $TRAIN --preset "$pn" $pa > "gpurun_out/preset_$pn.log" 2>&1 \
          || { tail -20 "gpurun_out/preset_$pn.log"; return 1; }
        echo "$pn: $(tail -1 "gpurun_out/preset_$pn.log" | cut -c1-400)"
      done ;;
    tuneplans)
      mkdir -p gpurun_out/plans
      rm -f gpurun_out/plans/cache.json
      for cmd in "python3 bench.py --steps 3 --warmup 5" "python3 bench.py --model vit_b16 --steps 3 --warmup 5" \
                 "python3 bench.py --model bert_large --steps 2 --warmup 3" \
                 "$TRAIN --preset bert_large_lamb --steps 1 --warmup_steps 2 --log_every 0"; do
        # shellcheck disable=SC2086
        DDL_GEMM_PLAN_TABLE=0 DDL_GEMM_TUNE_CACHE=gpurun_out/plans/cache.json timeout -k 10 400 $cmd \
          > gpurun_out/plans/tune.log 2>&1 || { tail -20 gpurun_out/plans/tune.log; return 1; }
        echo "$cmd: $(tail -1 gpurun_out/plans/tune.log | cut -c1-200)"
      done
      python3 -c "import json; print(len(json.load(open('gpurun_out/plans/cache.json'))), 'signatures')"
      # the BERT-large preset fits a larger batch once the table is loaded (no tuner workspaces in its
      # probe): after make_plan_table.py, run it again with the new table and add its misses with
      #   DDL_GEMM_TUNE_CACHE=gpurun_out/plans/preset_large.json $TRAIN --preset bert_large_lamb ...
      #   python scripts/make_plan_table.py --only-new gpurun_out/plans/preset_large.json
      ;;
    rehearse2)
      DDL_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --bert-batch 32 \
        > gpurun_out/rehearse2.log 2>&1 || { tail -30 gpurun_out/rehearse2.log; return 1; }
      tail -1 gpurun_out/rehearse2.log ;;
    script)
      local f=$1; shift
      timeout -k 10 300 python "$f" "$@" > "gpurun_out/script_$(basename "$f" .py).log" 2>&1 \
        || { tail -30 "gpurun_out/script_$(basename "$f" .py).log"; return 1; }
      tail -40 "gpurun_out/script_$(basename "$f" .py).log" ;;
    *) echo "unknown step $name" >&2; return 2 ;;
  esac
}

for s in "$@"; do
  # shellcheck disable=SC2086
  step $s || exit $?
done
