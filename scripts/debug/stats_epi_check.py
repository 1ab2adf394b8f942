"""Why does the narrow-kernel BN-statistics epilogue change z? Compare y / z / splits."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd import ops  # noqa: E402
from databricks_distributed_deep_learning_amd.ops import _native_conv as NC  # noqa: E402
from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG  # noqa: E402
from databricks_distributed_deep_learning_amd.ops.bridge import BNStats  # noqa: E402

dev = torch.device("cuda")
N, H, C, K, R, stride = 8, 28, 128, 512, 1, 1
torch.manual_seed(3)
x = torch.randn(N, H, H, C, device=dev).bfloat16()
w = (torch.randn(K, R, R, C, device=dev) * 0.1).bfloat16()
g = (torch.rand(K, device=dev) + 0.5).bfloat16()
b = torch.randn(K, device=dev).bfloat16()
NC.STATS_MIN_K = 0
NG.trace(True)
for kernel in ("narrow", "small", "big"):
    ys, zs = [], []
    for fused in (False, True):
        rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
        st = BNStats() if fused else None
        with NG.force_kernel(kernel):
            y = ops.conv2d(x, w, stride, R // 2, bn_stats=st)
        z = ops.batch_norm(y, g, b, rm, rv, True, 0.1, 1e-5, True, None, stats=st)
        ys.append(y.float())
        zs.append(z.float())
    recs = NG.trace(True)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    print(kernel, "launches", [(r[0][:4], r[1]) for r in recs],
          "y diff", (ys[0] - ys[1]).abs().max().item(), "y0 vs ref", (ys[0] - ref).abs().max().item(),
          "y1 vs ref", (ys[1] - ref).abs().max().item(),
          "z rel", ((zs[1] - zs[0]).abs().max() / zs[0].abs().max()).item(), flush=True)
