#!/usr/bin/env python3
"""ResNet stem (7x7 / stride-2 conv of the RGB image, 64 channels) on its space-to-depth form:
the direct kernels of csrc/kernels/stem_conv.hip against the implicit-GEMM path they replace.

    python benchmarks/stem_bench.py [--batch 256] [--image 224]

Per pass: median of 5 x 20 calls (HIP events), with the forward's BatchNorm statistics on, and
the bytes each pass must move at least (xs + y for the forward, xs + dy for the weight gradient)
as an effective TB/s.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, iters=20, reps=5):
    for _ in range(3):
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


class _Stats:
    def set(self, y, part, rows):
        pass


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    a = ap.parse_args()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    dev = torch.device("cuda")
    x = torch.randn(a.batch, a.image, a.image, 3, device=dev).to(torch.bfloat16)
    w = (torch.randn(64, 7, 7, 3, device=dev) * 0.1).to(torch.bfloat16)
    xs = NC._s2d_input(x, 3).contiguous()
    ws = NC._s2d_weight(w).contiguous()
    P, Q = xs.shape[1] - 3, xs.shape[2] - 3
    dy = torch.randn(a.batch, P, Q, 64, device=dev).to(torch.bfloat16)
    dw = torch.empty(64, 7, 7, 3, device=dev, dtype=torch.bfloat16)
    st = _Stats()
    fwd_bytes = xs.numel() * 2 + dy.numel() * 2
    rows = []
    for name, fn, nbytes in (
            ("fwd direct", lambda: NC._stem_fwd(xs, ws, st), fwd_bytes),
            ("fwd implicit GEMM", lambda: NC._fwd(xs, ws, 1, 0, stats=st), fwd_bytes),
            ("wgrad direct", lambda: NC._stem_wgrad(xs, dy, dw, accumulate=True), fwd_bytes),
            ("wgrad implicit GEMM", lambda: NC._wgrad(dy, xs, ws.shape, 1, 0), fwd_bytes)):
        ms = timeit(fn)
        rows.append({"pass": name, "us": round(ms * 1e3, 1), "min_bytes_TBps": round(nbytes / ms / 1e9, 2)})
        print(json.dumps({"batch": a.batch, "image": a.image, **rows[-1]}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
