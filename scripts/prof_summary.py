#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` database into per-kernel tables.

    python scripts/prof_summary.py gpurun_out/prof10/run_results.db --steps 8 \
        --split attn_fwd_k --names resnet50 bert_base > profiles/bench_kernels.md

``--split`` cuts the trace at the first dispatch whose name contains the given
substring (bench.py runs ResNet-50 first, then BERT-base: the first attention
kernel starts the second phase).  ``--steps`` divides totals to a per-step time
(warmup + timed steps that ran under the profiler).
"""
from __future__ import annotations

import argparse
import collections
import re
import sqlite3


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*$", "", name)
    return name[:90]


def load(db: str):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select name, start, end from kernels order by start").fetchall()
    return [(short(n), s, e) for n, s, e in rows]


def table(rows, steps: int, top: int, title: str) -> str:
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e in rows:
        agg[n][0] += e - s
        agg[n][1] += 1
    total = sum(v[0] for v in agg.values())
    out = [f"### {title}", "",
           f"GPU busy (sum of kernel time): {total / 1e6:.2f} ms total, {total / 1e6 / steps:.2f} ms/step "
           f"over {steps} profiled steps", "",
           "| kernel | calls/step | ms/step | avg us | % |", "|---|---:|---:|---:|---:|"]
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        out.append(f"| `{n}` | {c / steps:.1f} | {t / 1e6 / steps:.3f} | {t / c / 1e3:.1f} | {100 * t / total:.1f} |")
    return "\n".join(out) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--split", default=None)
    ap.add_argument("--names", nargs="*", default=["phase 1", "phase 2"])
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--after", default=None,
                    help="NAME:COUNT -- drop every dispatch up to and including the COUNT-th one whose name "
                         "contains NAME (e.g. sgd_k:3 skips 3 warm-up steps incl. the GEMM tuner's timing runs)")
    a = ap.parse_args()
    rows = load(a.db)
    if a.after:
        name, cnt = a.after.rsplit(":", 1)
        seen = 0
        for i, r in enumerate(rows):
            if name in r[0]:
                seen += 1
                if seen == int(cnt):
                    rows = rows[i + 1:]
                    break
    phases = [rows]
    if a.split:
        idx = next((i for i, r in enumerate(rows) if a.split in r[0]), len(rows))
        phases = [rows[:idx], rows[idx:]]
    for name, ph in zip(a.names, phases):
        if ph:
            print(table(ph, a.steps, a.top, name))


if __name__ == "__main__":
    main()
