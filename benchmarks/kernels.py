#!/usr/bin/env python3
"""Per-op microbenchmarks: our HIP kernels vs the stock PyTorch-ROCm path
(hipBLASLt GEMMs, MIOpen convs) on the exact shapes of the headline models.

    python benchmarks/kernels.py [--out results.json] [--only gemm|conv]

Timing: HIP events around 20 back-to-back calls after 5 warm-ups, median of 5
repeats, random bf16 operands (never zeros: MI355X clocks up on zero data).
"""
import argparse
import json
import statistics
import sys

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, iters=20, warm=5, reps=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) / iters)
    return statistics.median(out)


def bench_gemm(results):
    from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_NN, MODE_NT, MODE_TN, gemm
    dev = torch.device("cuda")
    T = 128 * 128
    shapes = [("qkv", T, 2304, 768), ("attn_out", T, 768, 768), ("ffn1", T, 3072, 768), ("ffn2", T, 768, 3072),
              ("sq4096", 4096, 4096, 4096)]
    for name, M, N, K in shapes:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
        NG.set_big_gemm(False)
        small = timeit(lambda: gemm(MODE_NT, a, K, w, K, c, N, M, N, K))
        NG.set_big_gemm(True)
        rows = {
            "fwd_ours128": small,
            "fwd_ours": timeit(lambda: gemm(MODE_NT, a, K, w, K, c, N, M, N, K)),
            "fwd_torch": timeit(lambda: torch.mm(a, w.t())),
            "dgrad_ours": timeit(lambda: gemm(MODE_NN, dy, N, w, K, dx, K, M, K, N)),
            "dgrad_torch": timeit(lambda: torch.mm(dy, w)),
            "wgrad_ours": timeit(lambda: gemm(MODE_TN, dy, N, a, K, dw, K, N, K, M)),
            "wgrad_torch": timeit(lambda: torch.mm(dy.t(), a)),
        }
        r = {"op": "gemm", "name": name, "M": M, "N": N, "K": K}
        for k, ms in rows.items():
            r[k + "_ms"] = round(ms, 4)
            r[k + "_tflops"] = round(fl / ms / 1e9, 1)
        results.append(r)
        print(json.dumps(r), flush=True)


def bench_conv(results, batch=256):
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    dev = torch.device("cuda")
    convs = [  # Cin, Cout, k, stride, H
        (3, 64, 7, 2, 224), (64, 64, 1, 1, 56), (64, 64, 3, 1, 56), (64, 256, 1, 1, 56), (256, 64, 1, 1, 56),
        (256, 128, 1, 1, 56), (128, 128, 3, 2, 56), (256, 512, 1, 2, 56), (128, 128, 3, 1, 28),
        (128, 512, 1, 1, 28), (512, 128, 1, 1, 28), (256, 256, 3, 1, 14), (256, 1024, 1, 1, 14),
        (1024, 256, 1, 1, 14), (512, 512, 3, 1, 7), (512, 2048, 1, 1, 7), (2048, 512, 1, 1, 7),
        (1024, 2048, 1, 2, 14), (512, 512, 3, 2, 14),
    ]
    for cin, cout, k, s, H in convs:
        pad = k // 2
        x = torch.randn(batch, H, H, cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(cout, k, k, cin, device=dev, dtype=torch.bfloat16) * 0.05
        P = (H + 2 * pad - k) // s + 1
        dy = torch.randn(batch, P, P, cout, device=dev, dtype=torch.bfloat16)
        xn = x.permute(0, 3, 1, 2)
        wn = w.permute(0, 3, 1, 2)
        dyn = dy.permute(0, 3, 1, 2)
        xp = F.pad(x, (0, (8 - cin % 8) % 8)) if cin % 8 else x
        wp = F.pad(w, (0, (8 - cin % 8) % 8)) if cin % 8 else w
        fl = 2.0 * batch * P * P * cout * k * k * cin
        r = {"op": "conv", "cin": cin, "cout": cout, "k": k, "stride": s, "H": H, "batch": batch}
        ops = {"fwd": lambda: NC._fwd(xp, wp, s, pad),
               "wgrad": lambda: NC._wgrad(dy, xp, wp.shape, s, pad)}
        ref = {"fwd": lambda: F.conv2d(xn, wn, stride=s, padding=pad),
               "wgrad": lambda: torch.ops.aten.convolution_backward(
                   dyn, xn, wn, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])}
        if cin % 8 == 0:
            ops["dgrad"] = lambda: NC._dgrad(dy, w, x.shape, s, pad)
            ref["dgrad"] = lambda: torch.ops.aten.convolution_backward(
                dyn, xn, wn, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False])
        for op, fn in ops.items():
            for kind in ("big", "small"):
                with NG.force_kernel(kind):
                    r[f"{op}_{kind}_ms"] = timeit(fn)
            r[f"{op}_tuned_ms"] = timeit(fn)
            r[f"{op}_miopen_ms"] = timeit(ref[op])
        for kk in list(r):
            if kk.endswith("_ms"):
                r[kk] = round(r[kk], 4)
                r[kk.replace("_ms", "_tflops")] = round(fl / r[kk] / 1e9, 1)
        results.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    res = []
    if a.only in ("", "gemm"):
        bench_gemm(res)
    if a.only in ("", "conv"):
        bench_conv(res, a.batch)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    sys.exit(0)
