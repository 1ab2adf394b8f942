set -o pipefail
mkdir -p gpurun_out/lnab
export TMPDIR=/tmp
NEW=$PWD/databricks_distributed_deep_learning_amd/_native/libddl_kernels.so
OLD=$PWD/databricks_distributed_deep_learning_amd/_native/ab/libddl_lnold.so
for i in 1 2; do
  for arm in new old; do
    if [ $arm = new ]; then export DDL_NATIVE_LIB=$NEW; else export DDL_NATIVE_LIB=$OLD; fi
    echo "$arm: $(timeout -k 10 120 python scripts/debug/ln_bwd_bench.py 2>/dev/null | tail -1)"
  done
done
for arm in new old; do
  if [ $arm = new ]; then export DDL_NATIVE_LIB=$NEW; else export DDL_NATIVE_LIB=$OLD; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS --output-format csv -d gpurun_out/lnab/$arm -o p -- python scripts/debug/ln_bwd_bench.py > gpurun_out/lnab/$arm.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for arm in ("new", "old"):
    tot = collections.defaultdict(float); n = set(); dur = 0.0
    for path in glob.glob(f"gpurun_out/lnab/{arm}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(path)):
            if "ln_bwd_k" not in row["Kernel_Name"]:
                continue
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            if row["Dispatch_Id"] not in n:
                n.add(row["Dispatch_Id"]); dur += (float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-3
    k = len(n)
    print(f"{arm}: {k} dispatches, {dur / k:.1f} us avg (profiled); per dispatch: LDS conflict cycles "
          f"{tot['SQ_LDS_BANK_CONFLICT'] / k:.0f}, LDS active cycles {tot['SQ_LDS_IDX_ACTIVE'] / k:.0f} "
          f"({100 * tot['SQ_LDS_BANK_CONFLICT'] / max(1, tot['SQ_LDS_IDX_ACTIVE']):.1f} %), LDS insts {tot['SQ_INSTS_LDS'] / k:.0f}, "
          f"wave cycles {tot['SQ_WAVE_CYCLES'] / k:.0f} (quad-cycles), busy cycles {tot['SQ_BUSY_CYCLES'] / k:.0f}")
PY
