"""BERT-base / ViT weight-gradient GEMMs on the dual-workgroup kernel with their planned split-K counts
(the split-K reduce included), accumulating into a bf16 gradient as in training; warm caches, median
of 30 launches: ``python scripts/debug/duo_tn_reduce_bench.py`` (DDL_NATIVE_LIB selects a library)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd.ops import _native_gemm as G  # noqa: E402

# (M = out features, N = in features, K = tokens, planned splits: ops/gemm_plans.json)
SHAPES = [(768, 768, 16384, 28), (2304, 768, 16384, 9), (3072, 768, 16384, 7), (768, 3072, 16384, 7),
          (768, 768, 25216, 28), (2304, 768, 25216, 9)]


def med_us(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in evs)
    return 1000.0 * t[len(t) // 2]


def main():
    dev = torch.device("cuda")
    lib = os.path.basename(os.environ.get("DDL_NATIVE_LIB", "tree"))
    for M, N, K, s in SHAPES:
        dy = torch.randn(K, M, device=dev).bfloat16()
        x = torch.randn(K, N, device=dev).bfloat16()
        dw = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        us = med_us(lambda: G.gemm(G.MODE_TN, dy, M, x, N, dw, N, M, N, K, accumulate=True, kernel="duo", splits=s))
        print(f"[{lib}] TN {M}x{N}x{K} duo x{s}: {us:.1f} us ({2 * M * N * K / us / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
