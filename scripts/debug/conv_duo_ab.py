"""ResNet-50 3x3 implicit-GEMM convolutions (batch 256) on each GEMM kernel kind, forced: the
forward with BatchNorm statistics and the input gradient with the BatchNorm-backward epilogue
(the shapes of profiles/gemm_trace_r50.md), cold-ish timings (50 back-to-back calls).

    python scripts/debug/conv_duo_ab.py [--kinds narrow big duo] [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG  # noqa: E402
from databricks_distributed_deep_learning_amd.ops._native_conv import _desc  # noqa: E402


def t_us(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", nargs="+", default=["narrow", "big", "duo"])
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda")
    Nb = a.batch
    # (H, W, C, K, stride): input spatial size, channels in / out
    for H, C, K, st in [(28, 128, 128, 1), (56, 128, 128, 2), (14, 256, 256, 1), (28, 256, 256, 2), (7, 512, 512, 1)]:
        x = torch.randn(Nb, H, H, C, device=dev).bfloat16()
        w = (torch.randn(K, 3, 3, C, device=dev) / (3 * C ** 0.5)).bfloat16()
        P = (H - 1) // st + 1
        M = Nb * P * P
        desc = _desc(Nb, H, H, C, P, P, st, -1, -1, 1, 1, 3, 3, P, P)
        y = torch.empty(M, K, device=dev).bfloat16()
        part = torch.empty(NG.stats_rows_max(M) * 2 * K + 64 * K, device=dev)
        xb = torch.randn(M, K, device=dev).bfloat16()
        mean, istd = torch.zeros(K, device=dev), torch.ones(K, device=dev)
        mask = torch.randint(0, 256, (M * K // 8,), device=dev, dtype=torch.uint8)
        fl = 2.0 * M * K * 9 * C
        row = [f"CONV {M}x{K}x{9 * C} (H={H}, C={C}, s={st})"]
        for kind in a.kinds:
            f = t_us(lambda: NG.gemm(NG.MODE_CONV, x, 0, w, 9 * C, y, K, M, K, 9 * C, conv=desc, colstats=part,
                                     kernel=kind))
            s = f"{kind}: stats {f:.1f} us ({fl / f / 1e6:.0f} TF)"
            if st == 1:
                b = t_us(lambda: NG.gemm(NG.MODE_CONV, x, 0, w, 9 * C, y, K, M, K, 9 * C, conv=desc, act="bnb",
                                         aux=xb, colstats=part, bnb=(mask, mean, istd), kernel=kind))
                s += f" bnb {b:.1f} ({fl / b / 1e6:.0f})"
            row.append(s)
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
