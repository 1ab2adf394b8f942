#!/usr/bin/env python3
"""1/2/4/8-GPU scaling sweep of the headline benchmark (BASELINE.json:2).

    python benchmarks/scaling.py [--ns 1,2,4,8] [--steps 20 --warmup 5] [--model both]
                                 [--native auto|stock] [--out scaling.json] [-- extra bench.py args]

Runs ``bench.py --gpus N`` once per N (capped at the visible GPU count; ``bench.py``
launches its N ranks itself), one N after another, and prints one JSON line per N
plus a summary with the weak-scaling efficiency of each N against N=1:

    efficiency(N) = value(N) / (N * value(1))     (per-GPU batch fixed: weak scaling)

Each run is a fresh set of processes: every N loads the committed GEMM plan table
(ops/gemm_plans.json; tuning only for a signature the table misses) and nothing from a
previous N is cached.  ``--backend gloo`` with
``--max-visible`` rehearses the sweep on the CPU
(tests/test_launch_cpu.py::test_bench_self_launch_and_scaling_sweep).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def visible_gpus() -> int:
    # device_count() does not initialise the GPU on this image (the parent stays GPU-free)
    import torch
    return torch.cuda.device_count()


def run_n(n: int, a, extra) -> dict:
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(a.steps),
           "--warmup", str(a.warmup), "--model", a.model, "--native", a.native] + list(extra)
    if a.backend:
        cmd += ["--backend", a.backend]
    t0 = time.time()
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=a.timeout)
    wall = time.time() - t0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"n_gpus": n, "ok": False, "rc": r.returncode, "wall_s": round(wall, 1)}
    rec = json.loads(lines[-1])
    rec.update(ok=True, wall_s=round(wall, 1))
    return rec


def efficiency(records) -> dict:
    base = next((r for r in records if r.get("ok") and r["n_gpus"] == 1), None)
    out = {}
    for r in records:
        if not r.get("ok") or base is None:
            continue
        n = r["n_gpus"]
        e = {"value": r["value"], "efficiency": round(r["value"] / (n * base["value"]), 4)}
        x, bx = r.get("extra", {}), base.get("extra", {})
        if "bert_base_samples_per_sec" in x and bx.get("bert_base_samples_per_sec"):
            e["bert_base_value"] = x["bert_base_samples_per_sec"]
            e["bert_base_efficiency"] = round(x["bert_base_samples_per_sec"] / (n * bx["bert_base_samples_per_sec"]), 4)
        out[str(n)] = e
    return out


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="both", choices=["both", "resnet50", "bert_base"])
    ap.add_argument("--native", default="auto", choices=["auto", "on", "off", "stock"])
    ap.add_argument("--backend", default="")
    ap.add_argument("--max-visible", type=int, default=0, help="cap N (CPU rehearsal: the visible 'devices')")
    ap.add_argument("--timeout", type=float, default=1800.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    cap = a.max_visible or visible_gpus() or 1
    ns = [n for n in (int(v) for v in a.ns.split(",")) if n <= cap]
    records = []
    for n in ns:
        rec = run_n(n, a, extra)
        print(json.dumps(rec), flush=True)
        records.append(rec)
    summary = {"sweep": "weak", "ns": ns, "native": a.native, "model": a.model, "efficiency": efficiency(records)}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"records": records, "summary": summary}, f, indent=1)
    return 0 if all(r.get("ok") for r in records) else 1


if __name__ == "__main__":
    sys.exit(main())
