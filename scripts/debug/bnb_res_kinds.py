"""Every kernel kind on ResNet-50's stage-4 BatchNorm-backward dgrad with a residual (NT 12544 x 2048 x 512,
``act="bnb"`` + residual + statistics partials: the one signature the plan table keeps on the 128x128 kernel),
isolated, cache-cold, device time: ``python scripts/debug/bnb_res_kinds.py``."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd.ops import _native_gemm as G  # noqa: E402


def t_us(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    buf = G._flush_buf(torch.cuda.current_device())
    evs = []
    for _ in range(reps):
        buf.fill_(1)
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
    for M, N, K, res in ((12544, 2048, 512, True), (12544, 2048, 512, False), (12544, 512, 2048, False)):
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(M, N, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16() if res else None
        mask = torch.randint(0, 256, (M * N // 8,), device=dev, dtype=torch.uint8)
        mean = torch.randn(N, device=dev)
        istd = torch.rand(N, device=dev) + 0.5
        part = torch.empty(G.stats_rows_max(M) * 2 * N, device=dev, dtype=torch.float32)
        cands = G._tune_candidates(G.MODE_NT, M, N, K, K, K, None, "bnb", x, False, r, part)
        out = []
        for kind, s in cands:
            try:
                us = t_us(lambda: G.gemm(G.MODE_NT, A, K, W, K, C, N, M, N, K, act="bnb", aux=x, residual=r,
                                         colstats=part, bnb=(mask, mean, istd), kernel=kind, splits=s))
                out.append(f"{kind}x{s} {us:.1f} us ({2 * M * N * K / us / 1e6:.0f} TF/s)")
            except Exception as e:       # noqa: BLE001
                out.append(f"{kind}x{s} failed: {str(e)[:80]}")
        print(f"NT {M}x{N}x{K} bnb{'+res' if res else ''}+stats: " + "; ".join(out), flush=True)
        if res:         # the same GEMM without the BatchNorm-backward epilogue, for scale
            for label, kw in (("plain", {}), ("+res", dict(residual=r)), ("+stats", dict(colstats=part))):
                out = []
                for kind in ("big", "small", "duo"):
                    try:
                        us = t_us(lambda: G.gemm(G.MODE_NT, A, K, W, K, C, N, M, N, K, kernel=kind, splits=1, **kw))
                        out.append(f"{kind} {us:.1f} us")
                    except Exception as e:       # noqa: BLE001
                        out.append(f"{kind} failed: {str(e)[:60]}")
                print(f"NT {M}x{N}x{K} {label}: " + "; ".join(out), flush=True)
            ew = torch.empty_like(x)
            print(f"elementwise x + r -> out (153 MB): {t_us(lambda: torch.add(x, r, out=ew)):.1f} us", flush=True)


if __name__ == "__main__":
    main()
