#!/usr/bin/env python3
"""Instruction census of the MFMA main loops in a kernel source (ISA level, no GPU needed).

    python scripts/isa_census.py csrc/kernels/gemm_duo.hip [--filter REGEX] [--asm OUT.s] [--min-mfma N]

Compiles the file for gfx950 to assembly (hipcc --cuda-device-only -S, the library's -O3 and the
MFMA VGPR-form flag of csrc/build.py where it applies), then for every kernel whose name matches
--filter finds its innermost loop holding >= 32 MFMAs (--min-mfma) (a back-edge branch to a label at or before
the branch) and counts the instructions by class: MFMA, VALU, SALU, LDS (ds_*), VMEM
(buffer / global, incl. LDS-DMA), plus the kernel's VGPR count and spill count.  VALU / MFMA in the
loop is what the per-MFMA-gap issue budget is spent on (MI355X_MICROARCH.md: a 16x16x32 MFMA gap
leaves ~8 free issue cycles; a wave64 VALU instruction issues over 2).
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_asm(src: str, out: str) -> None:
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    import build  # noqa: E402  (csrc/build.py: the library's per-file extra flags)
    extra = list(getattr(build, "EXTRA", {}).get(os.path.basename(src), []))
    cmd = ["hipcc", "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           "-I" + os.path.join(ROOT, "csrc", "include"), *extra, src, "-o", out]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def kernels(lines):
    """(name, body lines, metadata dict) per kernel in the assembly."""
    starts = [(i, m.group(1)) for i, l in enumerate(lines) if (m := re.match(r"^(_Z\S+):", l))]
    meta = {}
    name = None
    for l in lines:
        if (m := re.match(r"\s+\.name:\s+(\S+)", l)):
            name = m.group(1)
        for f in ("vgpr_count", "vgpr_spill_count", "sgpr_count"):
            if name and (m := re.match(r"\s+\." + f + r":\s+(\d+)", l)):
                meta.setdefault(name, {})[f] = int(m.group(1))
    for i, n in starts:
        j = i
        while j < len(lines) and not lines[j].strip().startswith(".Lfunc_end"):
            j += 1
        yield n, lines[i:j], meta.get(n, {})


def classify(op: str) -> str:
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "scratch_")):
        return "vmem"
    return "other"


def main_loop(body, min_mfma=32):
    labels = {b.split(":")[0]: j for j, b in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", b)}
    best = None
    for j, b in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch) (\.LBB\d+_\d+)", b)
        if not m or labels.get(m.group(1), 1 << 30) > j:
            continue
        lo = labels[m.group(1)]
        c = collections.Counter()
        for x in body[lo:j + 1]:
            t = x.strip().split()
            if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
                c[classify(t[0])] += 1
        # the innermost loop with the main loop's MFMAs: the shortest span holding >= 32 of them (a
        # persistent kernel's outer tile loop also holds the epilogue)
        if c["mfma"] >= min_mfma and (best is None or j - lo < best[2] - best[1]):
            best = (c, lo, j)
    return best


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default=".")
    ap.add_argument("--asm", default="")
    ap.add_argument("--min-mfma", type=int, default=32)
    a = ap.parse_args()
    out = a.asm or os.path.join(tempfile.mkdtemp(), "k.s")
    compile_asm(a.src, out)
    lines = open(out).read().split("\n")
    pat = re.compile(a.filter)
    print("| kernel | loop MFMA | VALU | SALU | LDS | VMEM | VALU/MFMA | VGPRs | spills |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for name, body, meta in kernels(lines):
        if not pat.search(name):
            continue
        r = main_loop(body, a.min_mfma)
        if r is None:
            continue
        c = r[0]
        demangled = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
        short = re.sub(r"\(anonymous namespace\)::", "", demangled).split("(")[0]
        print(f"| `{short}` | {c['mfma']} | {c['valu']} | {c['salu']} | {c['lds']} | {c['vmem']} | "
              f"{c['valu'] / c['mfma'] if c['mfma'] else float('nan'):.2f} | {meta.get('vgpr_count', '?')} | "
              f"{meta.get('vgpr_spill_count', '?')} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
