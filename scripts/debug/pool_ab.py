"""Time the ResNet stem's fused BN + ReLU + 3x3/2 max-pool forward and the max-pool backward at batch 256
(ddl_bn_relu_maxpool / ddl_maxpool_bwd), hot loop of back-to-back calls; DDL_POOL_XCD / DDL_POOL_BLOCK pick
the block order and size (A/B)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd.ops._lib import call, p  # noqa: E402


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


dev = torch.device("cuda")
N, H, W, C = 256, 112, 112, 64
P, Q = H // 2, W // 2
x = torch.randn(N, H, W, C, device=dev).bfloat16()
sc = torch.rand(C, device=dev) + 0.5
sh = torch.randn(C, device=dev) * 0.1
y = torch.empty(N, P, Q, C, device=dev, dtype=torch.bfloat16)
idx = torch.empty(N, P, Q, C, device=dev, dtype=torch.uint8)
mask = torch.empty(N * H * W * C // 8, device=dev, dtype=torch.uint8)
dy = torch.randn(N, P, Q, C, device=dev).bfloat16()
dx = torch.empty_like(x)
f = t_us(lambda: call("ddl_bn_relu_maxpool", 1, p(x), p(sc), p(sh), p(y), p(idx), p(mask), N, H, W, C, P, Q))
b = t_us(lambda: call("ddl_maxpool_bwd", 1, p(dy), p(idx), p(dx), N, H, W, C, P, Q, 3, 2, 1))
env = {k: v for k, v in os.environ.items() if k.startswith("DDL_POOL")}
print(f"{env} bn_relu_maxpool {f:.1f} us ({(411 + 103 + 51 + 51) / f * 1e-3:.2f} TB/s nominal)  "
      f"maxpool_bwd {b:.1f} us ({(411 + 103 + 51) / b * 1e-3:.2f} TB/s nominal)", flush=True)
