"""Time the LayerNorm backward (BERT-base shape, fused post-LN dropout) in isolation:
``python scripts/debug/ln_bwd_bench.py`` (grid knobs: DDL_LN_BWD_ROWS / DDL_LN_BWD_MAXBLK)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from databricks_distributed_deep_learning_amd import ops  # noqa: E402


def main():
    rows, H = 16384, 768
    dev = "cuda"
    x = torch.randn(rows, H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(rows, H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    b = torch.zeros(H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        y = ops.layer_norm(x, w, b, 1e-12, r, 0.1)
        y.backward(g)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    ys = [ops.layer_norm(x, w, b, 1e-12, r, 0.1) for _ in range(n)]
    e0.record()
    for y in ys:
        y.backward(g)
    e1.record()
    torch.cuda.synchronize()
    print(f"rows/blk={os.environ.get('DDL_LN_BWD_ROWS', '32')} cap={os.environ.get('DDL_LN_BWD_MAXBLK', '1024')} "
          f"ln backward {e0.elapsed_time(e1) / n * 1000:.1f} us")


if __name__ == "__main__":
    main()
