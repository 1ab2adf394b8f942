#!/usr/bin/env python3
"""Stage-1 1x1 conv GEMMs: the streaming skinny kernel (csrc/kernels/skinny_gemm.hip) vs the
tuned general kernels.   python benchmarks/skinny_bench.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.ops import _lib  # noqa: E402
from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_NT, gemm, stats_rows_max  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


GRID = int(__import__("os").environ.get("SK_GRID", "0"))


def main():
    dev = "cuda"
    M = 802816
    f = _lib.fn("ddl_skinny_gemm")
    for N, K in ((256, 64), (64, 256)):
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, N, device=dev).bfloat16()
        mask = torch.randint(0, 255, (M * N // 8,), device=dev, dtype=torch.uint8)
        mean, istd = torch.zeros(N, device=dev), torch.ones(N, device=dev)
        part = torch.empty(max(stats_rows_max(M), 1024) * 2 * N + 64 * 2 * N, device=dev)
        cases = {"stats": dict(stats=True), "res": dict(res=True)} if N == 256 else \
            {"stats": dict(stats=True), "bnb": dict(bnb=True, stats=True)}
        for name, o in cases.items():
            def sk():
                rc = f(a.data_ptr(), w.data_ptr(), c.data_ptr(), M, N, K, part.data_ptr() if o.get("stats") else 0,
                       res.data_ptr() if o.get("res") else 0, x.data_ptr() if o.get("bnb") else 0,
                       mask.data_ptr() if o.get("bnb") else 0, mean.data_ptr(), istd.data_ptr(), GRID, _lib.stream())
                assert rc >= 0, rc

            def gen():
                gemm(MODE_NT, a, K, w, K, c, N, M, N, K, residual=res if o.get("res") else None,
                     colstats=part if o.get("stats") else None, act="bnb" if o.get("bnb") else None,
                     aux=x if o.get("bnb") else None, bnb=(mask, mean, istd) if o.get("bnb") else None)
            print(json.dumps({"N": N, "K": K, "case": name, "skinny_us": round(timeit(sk), 1),
                              "general_us": round(timeit(gen), 1)}))


if __name__ == "__main__":
    main()
