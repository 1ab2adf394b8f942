#!/usr/bin/env python3
"""Per-kernel hardware-counter table from ``scripts/pmc_profile.sh`` output.

    python scripts/pmc_summary.py gpurun_out/pmc_gemm [--top 25] [--match gemm] > profiles/pmc_gemm.md

Reads every ``*counter_collection.csv`` under the directory (one row per dispatch and
counter), sums each counter per kernel name and derives:

* MFMA busy %   = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs ... ) -- reported
  as MFMA cycles per CU-cycle: busy / (GRBM_GUI_ACTIVE * CUs * 4 SIMDs);
* wave-time split = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES;
* LDS bank-conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* HBM bytes = 2 * FETCH_SIZE (gfx950 FETCH_SIZE counts half of a wide coalesced
  stream, see MI355X_MICROARCH.md section HBM) + WRITE_SIZE, in KB units; GB/s over the
  kernel's summed duration from the same pass;
* L2 hit % = TCC_HIT / (TCC_HIT + TCC_MISS).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re

NUM_CU = 256


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*$", "", name)
    return name[:80]


def steady_ids(rows, after: str):
    """Dispatch ids past the N-th dispatch of the kernel named in ``after`` ("name:N", e.g. the
    optimizer kernel that ends each warm-up step): the warm-up steps' dispatches are dropped."""
    if not after:
        return None
    name, _, n = after.rpartition(":")
    order = {}
    for row in rows:
        did = int(row.get("Dispatch_Id") or 0)
        order.setdefault(did, short(row.get("Kernel_Name", "?")))
    seen = 0
    for did in sorted(order):
        if name in order[did]:
            seen += 1
            if seen == int(n):
                return {d for d in order if d > did}
    return set()


def load(d: str, after: str = ""):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(lambda: collections.defaultdict(float))   # per pass file
    calls = collections.defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        with open(path) as f:
            rows = list(csv.DictReader(f))
        keep = steady_ids(rows, after)
        if True:
            for row in rows:
                if keep is not None and int(row.get("Dispatch_Id") or 0) not in keep:
                    continue
                k = short(row.get("Kernel_Name", "?"))
                vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
                did = (path, row.get("Dispatch_Id"))
                calls[k].add(did)
                if did not in seen and row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    seen.add(did)
                    dur[k][path] += (float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-9
    return vals, dur, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--match", default="")
    ap.add_argument("--title", default="")
    ap.add_argument("--after", default="", help="name:N -- count only dispatches after the N-th dispatch of "
                                                "kernel `name` (drop the warm-up steps)")
    a = ap.parse_args()
    vals, dur, calls = load(a.dir, a.after)
    names = [k for k in vals if a.match in k]
    tot_t = {k: max(dur[k].values()) if dur[k] else 0.0 for k in names}
    names.sort(key=lambda k: -tot_t[k])
    print(f"### {a.title or a.dir}\n")
    print("MFMA% = MFMA-busy cycles per SIMD-cycle while the GPU was active; wave time = "
          "waiting (s_waitcnt/barrier) / issue-stalled / issuing, as % of SQ_WAVE_CYCLES; "
          "HBM = 2*FETCH_SIZE + WRITE_SIZE.\n")
    print("| kernel | dispatches | time ms | MFMA % | wait % | stall % | issue % | LDS confl % | "
          "HBM GB | HBM GB/s | L2 hit % | VALU/MFMA insts |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in names[:a.top]:
        v = vals[k]
        t = tot_t[k]
        gact = v.get("GRBM_GUI_ACTIVE", 0.0)
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy over all 1024 SIMDs
        mfma = 100.0 * v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gact / 8 * NUM_CU * 4) if gact else float("nan")
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        pct = (lambda c: 100.0 * v.get(c, 0.0) / wc if wc else float("nan"))
        lds = v.get("SQ_LDS_IDX_ACTIVE", 0.0)
        confl = 100.0 * v.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else float("nan")
        hbm = (2 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0)) * 1024 / 1e9
        hit, miss = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
        l2 = 100.0 * hit / (hit + miss) if hit + miss else float("nan")
        mi = v.get("SQ_INSTS_MFMA", 0.0)
        vr = v.get("SQ_INSTS_VALU", 0.0) / mi if mi else float("nan")
        ncall = len(calls[k]) // 3 if len(calls[k]) >= 3 else len(calls[k])
        print(f"| `{k}` | {ncall} | {t * 1e3:.3f} | {mfma:.1f} | {pct('SQ_WAIT_ANY'):.1f} | "
              f"{pct('SQ_WAIT_INST_ANY'):.1f} | {pct('SQ_ACTIVE_INST_ANY'):.1f} | {confl:.2f} | {hbm:.3f} | "
              f"{hbm / t if t else float('nan'):.0f} | {l2:.1f} | {vr:.2f} |")


if __name__ == "__main__":
    main()
