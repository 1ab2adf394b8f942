"""Time the BatchNorm statistics finalize (norm.hip bn_fwd_finalize_k, fed from GEMM-epilogue
partial rows) on every ResNet-50 (batch 256) BatchNorm shape, back-to-back launches replayed from one HIP graph:
``python scripts/debug/fin_bench.py``.  A tiny launch (bn_eval_coeffs_k, C = 64) gives the
per-launch floor of the same loop."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from databricks_distributed_deep_learning_amd.ops._lib import call, p  # noqa: E402

# (M, C, BatchNorm layers of that shape per step) for ResNet-50 at batch 256, 224 x 224
# (a stage's first bottleneck has its 1x1 reduction BN at the previous stage's resolution: stride on the 3x3)
SHAPES = [(3211264, 64, 1), (802816, 64, 6), (802816, 256, 4), (802816, 128, 1), (200704, 128, 7),
          (200704, 512, 5), (200704, 256, 1), (50176, 256, 11), (50176, 1024, 7), (50176, 512, 1),
          (12544, 512, 5), (12544, 2048, 4)]


def timed(fn, n=100):
    """GPU time per launch: n launches captured in one graph (host launch cost out of the loop)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(n):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * n) * 1000.0


def main():
    dev = "cuda"
    f32 = dict(dtype=torch.float32, device=dev)
    g = torch.ones(2048, dtype=torch.bfloat16, device=dev)
    b = torch.zeros(2048, dtype=torch.bfloat16, device=dev)
    rm, rv = torch.zeros(2048, **f32), torch.ones(2048, **f32)
    stats = torch.empty(4, 2048, **f32)
    floor = timed(lambda: call("ddl_bn_eval_coeffs", 1, 64, p(g), p(b), p(rm), p(rv), 1e-5, p(stats[2]),
                               p(stats[3])))
    print(f"launch floor (bn_eval_coeffs_k, C=64): {floor:.2f} us")
    total = 0.0
    for M, C, count in SHAPES:
        nblk = -(-M // 128)
        part = torch.rand(nblk * 2 * C, **f32)
        ws = torch.empty(-(-nblk // 32) * 2 * C, **f32)
        st = torch.empty(4, C, **f32)

        def run():
            call("ddl_bn_fwd_from_partials", 1, p(part), nblk, M, C, p(g), p(b), p(rm), p(rv), 0.1, 1e-5,
                 p(st[0]), p(st[1]), p(st[2]), p(st[3]), p(ws), ws.numel())
        us = timed(run)
        mb = nblk * 2 * C * 4 / 1e6
        total += us * count
        print(f"M={M:8d} C={C:5d} rows={nblk:6d} x{count:2d}: {us:6.2f} us/launch  {mb:7.2f} MB  "
              f"{mb / us * 1e3:7.0f} GB/s")
    print(f"forward finalize per step (53 layers): {total:.1f} us")


if __name__ == "__main__":
    main()
