"""Register-spill check for the hand-written GEMM kernels (profiles/gemm_spills_r04.md).

Emits the gfx950 device assembly of a kernel source (``hipcc --cuda-device-only -S``, ~4 min for
gemm_big.hip) or reads an existing ``.s`` and reports, per ``gemm_big_k`` instantiation and for ``gemm_wg_k``, the scratch
(spill) instructions in the whole body and inside its MFMA main loop (the span between the first and
last ``v_mfma`` of the densest cluster).  Exits 1 if any main loop holds more than ``--max-loop``.

    python scripts/check_spills.py                      # compile csrc/kernels/gemm_big.hip
    python scripts/check_spills.py --asm /tmp/gb.s      # scan an existing assembly file
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"\n(_ZN\w*gemm_(?:big|wg)_k\w*):[^\n]*\n(.*?)\.Lfunc_end", re.S)
TPL = re.compile(r"gemm_big_kILi(\d)ELi(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)E")


def emit(src: str, out: str, defines) -> None:
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I",
           os.path.join(ROOT, "csrc", "include"), "-ffp-contract=fast", "-munsafe-fp-atomics", "-x", "hip",
           "--cuda-device-only", "-S", src, "-o", out] + [f"-D{d}" for d in defines]
    if os.path.basename(src) == "gemm_big.hip":     # the library's flags for it (csrc/build.py EXTRA)
        cmd += ["-mllvm", "-amdgpu-mfma-vgpr-form"]
    subprocess.run(cmd, check=True)


def scan(text: str):
    rows = []
    for m in PAT.finditer(text):
        name, body = m.group(1), m.group(2)
        t = TPL.search(name)
        tag = "".join(t.groups()) if t else "wg" if "gemm_wg_k" in name else name[-40:]
        lines = body.split("\n")
        mf = [i for i, ln in enumerate(lines) if "v_mfma" in ln]
        sc = [i for i, ln in enumerate(lines) if "scratch_" in ln]
        loop = 0
        if mf:
            # MFMA clusters: runs of v_mfma lines less than 400 lines apart; the main loop is the largest
            clusters, a, prev = [], mf[0], mf[0]
            for i in mf[1:]:
                if i - prev > 400:
                    clusters.append((a, prev))
                    a = i
                prev = i
            clusters.append((a, prev))
            lo, hi = max(clusters, key=lambda c: sum(1 for x in mf if c[0] <= x <= c[1]))
            loop = sum(1 for i in sc if lo <= i <= hi)
        rows.append((tag, len(mf), len(sc), loop))
    return rows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default="")
    ap.add_argument("--src", default=os.path.join(ROOT, "csrc", "kernels", "gemm_big.hip"))
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--max-loop", type=int, default=16)
    a = ap.parse_args()
    path = a.asm
    if not path:
        path = os.path.join(tempfile.mkdtemp(), "k.s")
        emit(a.src, path, a.defines)
    with open(path) as f:
        rows = scan(f.read())
    bad = 0
    print("instantiation <LA LB KTAIL DIRECT BNB EDGE N192>  mfma  scratch  scratch-in-main-loop")
    for tag, nmf, nsc, loop in rows:
        flag = "  <-- spills in the main loop" if loop > a.max_loop else ""
        bad += bool(flag)
        print(f"{tag:>10} {nmf:6d} {nsc:8d} {loop:8d}{flag}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
