#!/usr/bin/env python3
"""Stage-1 ResNet-50 3x3 conv (256 x 56 x 56 x 64 -> 64): direct kernel vs implicit GEMM.
    python benchmarks/conv3x3_bench.py [--grid G ...]"""
import argparse
import json
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.ops import _native_conv as nc  # noqa: E402
from databricks_distributed_deep_learning_amd.ops.bridge import BNStats  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs="*", default=[0, 512, 1024])
    ap.add_argument("--n", type=int, default=256)
    a = ap.parse_args()
    N, H, W = a.n, 56, 56
    x = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    w = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).bfloat16()
    y = torch.empty_like(x)
    part = torch.empty(nc._direct3x3_rows(N * H * W) * 128, device="cuda")
    aux = torch.randn_like(x)
    mask = torch.randint(0, 255, (x.numel() // 8,), device="cuda", dtype=torch.uint8)
    hint = SimpleNamespace(x=aux, mask=mask, mean=torch.zeros(64, device="cuda"), istd=torch.ones(64, device="cuda"),
                           set=lambda *args: None)
    dw = torch.empty(64, 3, 3, 64, device="cuda", dtype=torch.bfloat16)
    out = {}
    for g in a.grid:
        out[f"direct_fwd_stats_g{g}"] = timeit(lambda: nc._direct3x3(x, w, y, part, grid=g))
        out[f"direct_dgrad_bnb_g{g}"] = timeit(lambda: nc._direct3x3(x, w, y, part, bnb=hint, grid=g))
        out[f"direct_fwd_plain_g{g}"] = timeit(lambda: nc._direct3x3(x, w, y, None, grid=g))
        out[f"direct_wgrad_g{g}"] = timeit(lambda: nc._direct3x3_wgrad(aux, x, dw, False, grid=g))
    nc._CONV3X3 = False
    st = BNStats()
    out["gemm_fwd_stats"] = timeit(lambda: nc._fwd(x, w, 1, 1, stats=st))
    out["gemm_fwd_plain"] = timeit(lambda: nc._fwd(x, w, 1, 1))
    out["gemm_dgrad_bnb"] = timeit(lambda: nc._dgrad(x, w, x.shape, 1, 1, bnb=hint))
    out["gemm_dgrad_plain"] = timeit(lambda: nc._dgrad(x, w, x.shape, 1, 1))
    out["gemm_wgrad"] = timeit(lambda: nc._wgrad(aux, x, w.shape, 1, 1))
    nc._CONV3X3 = True
    for k, v in out.items():
        print(json.dumps({"case": k, "us": round(v, 1)}))


if __name__ == "__main__":
    main()
