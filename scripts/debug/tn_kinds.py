"""Time every tuner candidate of the BERT-base weight-gradient GEMMs (TN, K = tokens) in isolation,
operands cache-hot and from an evicted cache, accumulating into a bf16 gradient like the model does.
DDL_NATIVE_LIB picks the library build (A/B of kernel variants)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd.ops import _native_gemm as G  # noqa: E402


def t_us(fn, reps=20, cold=False):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    buf = G._flush_buf(torch.cuda.current_device()) if cold else None
    evs = []
    torch.cuda._sleep(int(3e5 * reps))
    for _ in range(reps):
        if cold:
            buf.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in evs)
    return 1000.0 * t[len(t) // 2]


dev = torch.device("cuda")
T = int(os.environ.get("TN_T", "16384"))
lib = os.path.basename(os.environ.get("DDL_NATIVE_LIB", "default"))
for N, K in [(2304, 768), (3072, 768), (768, 3072), (768, 768)]:
    dy = torch.randn(T, N, device=dev).bfloat16()
    x = torch.randn(T, K, device=dev).bfloat16()
    g = torch.zeros(N, K, device=dev).bfloat16()
    cands = G._tune_candidates(G.MODE_TN, N, K, T, N, K, None, None, None, False, None, None)
    row = []
    for kind, s in cands:
        fn = lambda kind=kind, s=s: G._launch(kind, s, G.MODE_TN, dy, N, x, K, g, K, N, K, T, None, None,  # noqa: E731
                                              None, None, False, None, True)
        hot, cold = t_us(fn), t_us(fn, cold=True)
        row.append(f"{kind}:{s} {hot:.1f}/{cold:.1f}")
    print(f"[{lib}] TN {N}x{K}x{T} (hot/cold us): " + "  ".join(row), flush=True)
