#!/usr/bin/env python3
"""Stage-2 / 3 1x1 conv GEMMs (M = 200704 = 256 x 28 x 28 / 50176 = 256 x 14 x 14): the register-B streaming kernel
(csrc/kernels/stream_gemm.hip) vs the tuned general kernels, with the epilogues the ResNet-50
step runs (statistics, BN-backward, residual + BN-backward).  Effective TB/s = the bytes the
GEMM must move (operands, epilogue inputs, output) over its time.
    python benchmarks/stream_bench.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.ops import _lib  # noqa: E402
from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_NT, gemm, stats_rows_max  # noqa: E402


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
    dev = "cuda"
    f = _lib.fn("ddl_stream_gemm")
    for N, K, M in ((512, 128, 200704), (128, 512, 200704), (1024, 256, 50176), (256, 1024, 50176)):
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, N, device=dev).bfloat16()
        mask = torch.randint(0, 255, (M * N // 8,), device=dev, dtype=torch.uint8)
        mean, istd = torch.zeros(N, device=dev), torch.ones(N, device=dev)
        part = torch.empty(max(stats_rows_max(M), 1024) * 2 * N + 64 * 2 * N, device=dev)
        cases = {"stats": dict(stats=True), "bnb": dict(bnb=True, stats=True)}
        if N in (512, 1024):
            cases["res,bnb"] = dict(res=True, bnb=True, stats=True)
        for name, o in cases.items():
            def st():
                rc = f(a.data_ptr(), w.data_ptr(), c.data_ptr(), M, N, K, part.data_ptr(),
                       res.data_ptr() if o.get("res") else 0, x.data_ptr() if o.get("bnb") else 0,
                       mask.data_ptr() if o.get("bnb") else 0, mean.data_ptr(), istd.data_ptr(), 0, _lib.stream())
                assert rc >= 0, rc

            def gen():
                gemm(MODE_NT, a, K, w, K, c, N, M, N, K, residual=res if o.get("res") else None,
                     colstats=part, act="bnb" if o.get("bnb") else None,
                     aux=x if o.get("bnb") else None, bnb=(mask, mean, istd) if o.get("bnb") else None)
            nbytes = 2 * M * (K + N) + (2 * M * N if o.get("res") else 0) + (2 * M * N + M * N // 8 if o.get("bnb") else 0)
            ts, tg = timeit(st), timeit(gen)
            print(json.dumps({"N": N, "K": K, "case": name, "stream_us": round(ts, 1), "general_us": round(tg, 1),
                              "stream_TBps": round(nbytes / ts / 1e6, 2), "general_TBps": round(nbytes / tg / 1e6, 2)}))


def wgrad():
    """TN weight gradients of the ResNet-50 1x1 convs: the streaming kernel ("swg") against the
    tuner's other candidates (cold-cache timing, as the tuner sees them)."""
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    dev = "cuda"
    for M, N, K in ((256, 64, 802816), (64, 256, 802816), (64, 64, 802816), (128, 256, 802816),
                    (512, 128, 200704), (128, 512, 200704), (256, 512, 200704)):
        a = torch.randn(K, M, device=dev).bfloat16()
        b = torch.randn(K, N, device=dev).bfloat16()
        c = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        res = {}
        for kind, s in NG._candidates(NG.MODE_TN, M, N, K, False, M, N, plain=True):
            if s == 1 and kind in ("big", "small", "narrow", "tnarrow"):
                continue      # unsplit: a single round of tiles, far off
            res[f"{kind}:{s}"] = round(timeit(lambda: NG._launch(kind, s, NG.MODE_TN, a, M, b, N, c, N, M, N, K, None,
                                                                 None, None, None, False, None, True)), 1)
        nbytes = 2 * K * (M + N)
        best = min(res, key=res.get)
        print(json.dumps({"TN": [M, N, K], "us": res, "best": best, "best_TBps": round(nbytes / res[best] / 1e6, 2)}))


if __name__ == "__main__":
    main()
    wgrad()
