#!/usr/bin/env python3
"""Refresh the committed GEMM kernel plan table (``ops/gemm_plans.json``) from tuning runs.

    python scripts/make_plan_table.py [--arch gfx950] [--replace] CACHE.json [CACHE.json ...]

Each CACHE is a ``DDL_GEMM_TUNE_CACHE`` file written by a tuning run on the GPU (the isolated
cold-cache tuner for CNN shapes, the in-model tuner for transformer shapes), e.g.

    DDL_GEMM_PLAN_TABLE=0 DDL_GEMM_TUNE_CACHE=gpurun_out/plans/r50.json python bench.py --model resnet50

The table entry for ``--arch`` is keyed by the hash of the GEMM kernel sources the in-tree library
was built from (``csrc/build.py`` gemm_src_hash): entries tuned against other sources are dropped
(``--replace`` drops every old entry), later CACHE files override earlier ones signature by
signature.  Runs on the CPU: it only reads the library's recorded hash.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "csrc"))
TABLE = os.path.join(ROOT, "databricks_distributed_deep_learning_amd", "ops", "gemm_plans.json")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("caches", nargs="+")
    ap.add_argument("--arch", default="gfx950")
    ap.add_argument("--replace", action="store_true", help="drop the architecture's old entries first")
    ap.add_argument("--table", default=TABLE)
    ap.add_argument("--only-new", action="store_true", help="add signatures the table lacks; keep existing entries")
    a = ap.parse_args()
    import build as native_build     # csrc/build.py: the same hash the library embeds
    src = native_build.gemm_src_hash()
    from databricks_distributed_deep_learning_amd.ops import _lib
    built = _lib.gemm_src_hash()
    if built is not None and built != src:
        print(f"warning: the built library has GEMM source hash {built}, the tree {src}: rebuild first",
              file=sys.stderr)
        return 1
    doc = {}
    if os.path.exists(a.table):
        with open(a.table) as f:
            doc = json.load(f)
    ent = doc.get(a.arch, {})
    plans = {} if a.replace or ent.get("gemm_src_hash") != src else dict(ent.get("plans", {}))
    n0 = len(plans)
    for path in a.caches:
        with open(path) as f:
            for k, v in json.load(f).items():
                if a.only_new and k in plans:
                    continue
                plans[k] = [str(v[0]), int(v[1])]
    doc[a.arch] = {"gemm_src_hash": src, "plans": dict(sorted(plans.items()))}
    with open(a.table + ".tmp", "w") as f:      # one line per signature (reviewable diffs)
        f.write("{\n")
        for ai, arch in enumerate(sorted(doc)):
            ent = doc[arch]
            f.write(f' {json.dumps(arch)}: {{\n  "gemm_src_hash": {json.dumps(ent["gemm_src_hash"])},\n  "plans": {{\n')
            items = sorted(ent["plans"].items())
            for i, (k, v) in enumerate(items):
                f.write(f"   {json.dumps(k)}: {json.dumps(v)}{',' if i + 1 < len(items) else ''}\n")
            f.write(f"  }}\n }}{',' if ai + 1 < len(doc) else ''}\n")
        f.write("}\n")
    os.replace(a.table + ".tmp", a.table)
    print(f"{a.table}: {a.arch} @ {src}: {len(plans)} signatures ({n0} kept, {len(plans) - n0} added; later files override "
          f"from {len(a.caches)} file(s))")
    return 0


if __name__ == "__main__":
    sys.exit(main())
