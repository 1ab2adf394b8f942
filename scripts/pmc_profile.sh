#!/bin/bash
# rocprofv3 hardware-counter passes ("rocprof counters shown").
# Each pass is its own short run (rocprofv3 does not split counters over passes;
# per-pass slots on gfx950: 8 SQ, 4 TCC, 2 GRBM), counters only with
# --kernel-trace, never with sys/runtime traces.
#
#   scripts/pmc_profile.sh <outdir> -- <program> [args...]
#   python scripts/pmc_summary.py <outdir> > profiles/pmc_<name>.md
set -o pipefail
out="$1"; shift
[ "$1" = "--" ] && shift
mkdir -p "$out"
export TMPDIR=/tmp
# pass 1: where wave time goes (quad-cycles) + MFMA busy (cycles) + LDS
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
# pass 2: HBM read bytes (FETCH_SIZE: 3 TCC slots) + GPU clock
P2="FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
# pass 3: HBM write bytes (WRITE_SIZE: 2 slots) + L2 hit / miss
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for pmc in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  echo "=== pmc pass $i: $pmc" >&2
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d "$out/pass$i" -o pass$i -- "$@" \
    > "$out/pass$i.log" 2>&1
  rc=$?
  echo "=== pmc pass $i rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -20 "$out/pass$i.log" >&2; exit $rc; fi
done
exit 0
