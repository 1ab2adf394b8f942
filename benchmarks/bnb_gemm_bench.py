#!/usr/bin/env python3
"""dgrad GEMM with the BatchNorm-backward epilogue (+ residual): the residual-block shapes
of ResNet-50, per kernel family.   python benchmarks/bnb_gemm_bench.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_NT, gemm, stats_rows_max  # noqa: E402

SHAPES = [(802816, 256, 64), (200704, 512, 128), (50176, 1024, 256), (12544, 2048, 512)]


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


def main():
    dev = "cuda"
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(M, N, device=dev).bfloat16()
        res = torch.randn(M, N, device=dev).bfloat16()
        mask = torch.randint(0, 255, (M * N // 8,), device=dev, dtype=torch.uint8)
        mean, istd = torch.zeros(N, device=dev), torch.ones(N, device=dev)
        rows = stats_rows_max(M)
        part = torch.empty((rows + rows // 32 + 1) * 2 * N, device=dev)
        gb = (M * K * 2 + 3 * M * N * 2 + M * N // 8) / 1e9
        for kern in ("small", "big"):
            for with_res in (False, True):
                def run():
                    gemm(MODE_NT, a, K, w, K, c, N, M, N, K, act="bnb", aux=x, residual=res if with_res else None,
                         colstats=part, bnb=(mask, mean, istd), kernel=kern)
                try:
                    us = timeit(run)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"shape": [M, N, K], "kernel": kern, "res": with_res, "error": str(e)[:80]}))
                    continue
                g = gb + (M * N * 2 / 1e9 if with_res else 0)
                print(json.dumps({"shape": [M, N, K], "kernel": kern, "res": with_res, "us": round(us, 1),
                                  "TB/s": round(g / us * 1e6 / 1e3, 2)}))
        def plain():
            gemm(MODE_NT, a, K, w, K, c, N, M, N, K, residual=res)
        us = timeit(plain)
        print(json.dumps({"shape": [M, N, K], "kernel": "auto", "plain_res": True, "us": round(us, 1)}))


if __name__ == "__main__":
    main()
