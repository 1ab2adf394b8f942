#!/usr/bin/env python3
"""Build the native kernel library for gfx950 (MI355X).

    python csrc/build.py [--clean] [-j N] [--debug]

Compiles every ``csrc/kernels/*.hip`` and ``csrc/runtime/*.cpp`` with
``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU) into
``databricks_distributed_deep_learning_amd/_native/libddl_kernels.so``: one
shared object with a plain C ABI, loaded by ``ops/_lib.py`` via ctypes.  No
torch headers are involved, so a full rebuild takes seconds, and objects are
rebuilt only when a source or header is newer than its object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
OUT_DIR = os.path.join(ROOT, "databricks_distributed_deep_learning_amd", "_native")
OUT = os.path.join(OUT_DIR, "libddl_kernels.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DDL_OFFLOAD_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(CSRC, "include"),
          "-Wno-unused-result", "-ffp-contract=fast", "-munsafe-fp-atomics"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))) + \
        sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))


def headers():
    return glob.glob(os.path.join(CSRC, "include", "*.h")) + glob.glob(os.path.join(CSRC, "kernels", "*.h"))


def obj_for(src):
    return os.path.join(BUILD, os.path.basename(src) + ".o")


def needs(src, obj, hdr_mtime):
    if not os.path.exists(obj):
        return True
    m = os.path.getmtime(obj)
    return os.path.getmtime(src) > m or hdr_mtime > m


# per-source extra flags: the VGPR form of the MFMA instructions.  With AGPR-form accumulators the
# allocator shuffled them through v_accvgpr moves around the MFMAs: gemm_big.hip's 4-wave weight-
# gradient kernel (2.7x its MFMA time), conv3x3_wgrad_k (620 moves per 144 MFMAs, 414 registers ->
# 260), the skinny GEMMs.  gemm_big.hip's 8-wave kernels compile identically either way.
_VGPR_FORM = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
EXTRA = {"gemm_big.hip": _VGPR_FORM, "conv3x3.hip": _VGPR_FORM, "skinny_gemm.hip": _VGPR_FORM,
         "stream_gemm.hip": _VGPR_FORM, "gemm_duo.hip": _VGPR_FORM}


# Sources whose code decides which GEMM kernel runs fastest for a shape: their hash keys the committed
# kernel plan table (ops/gemm_plans.json) -- a plan tuned against other GEMM kernels is not used.
GEMM_SOURCES = ["gemm.hip", "gemm_big.hip", "gemm_duo.hip", "skinny_gemm.hip", "stream_gemm.hip", "conv3x3.hip"]


def gemm_src_hash() -> str:
    import hashlib
    h = hashlib.sha256()
    for name in GEMM_SOURCES + ["../include/ddl_common.h"]:
        path = os.path.normpath(os.path.join(CSRC, "kernels", name))
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def buildinfo_obj() -> str:
    """A host object exporting ddl_gemm_src_hash() (rebuilt whenever that hash changes)."""
    digest = gemm_src_hash()
    src = os.path.join(BUILD, "buildinfo.cpp")
    obj = src + ".o"
    text = ('extern "C" __attribute__((visibility("default"))) const char* ddl_gemm_src_hash() '
            f'{{ return "{digest}"; }}\n')
    old = open(src).read() if os.path.exists(src) else ""
    if old != text or not os.path.exists(obj):
        with open(src, "w") as f:
            f.write(text)
        r = subprocess.run(["g++", "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"buildinfo compile failed: {r.stderr}")
    return obj


def compile_one(src, debug=False):
    obj = obj_for(src)
    flags = list(COMMON) + EXTRA.get(os.path.basename(src), [])
    if debug:
        flags = [f for f in flags if f != "-O3"] + ["-O1", "-g"]
    if src.endswith(".cpp"):
        flags += ["-x", "hip"]
    cmd = [HIPCC, *flags, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int = 8, clean: bool = False, debug: bool = False, verbose: bool = True) -> str:
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    srcs = sources()
    if not srcs:
        raise RuntimeError("no native sources found under csrc/")
    hm = max([os.path.getmtime(h) for h in headers()] + [0.0])
    todo = [s for s in srcs if needs(s, obj_for(s), hm)]
    if verbose:
        print(f"[build] {len(todo)}/{len(srcs)} sources to compile for {ARCH}", file=sys.stderr)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(compile_one, s, debug): s for s in todo}
        for f in cf.as_completed(futs):
            f.result()
            if verbose:
                print(f"[build]   ok {os.path.relpath(futs[f], ROOT)}", file=sys.stderr)
    objs = [obj_for(s) for s in srcs] + [buildinfo_obj()]
    newest = max(os.path.getmtime(o) for o in objs)
    if todo or not os.path.exists(OUT) or os.path.getmtime(OUT) < newest:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT + ".tmp",
               "-L/opt/rocm/lib", "-Wl,--no-as-needed", "-lamdhip64", "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(OUT + ".tmp", OUT)
        if verbose:
            print(f"[build] linked {os.path.relpath(OUT, ROOT)}", file=sys.stderr)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args()
    build(a.jobs, a.clean, a.debug)
