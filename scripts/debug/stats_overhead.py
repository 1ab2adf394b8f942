"""Cost of the BN-statistics GEMM epilogue per conv shape and kernel (GPU debugging aid)."""
import sys

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.ops import _native_conv as NC  # noqa: E402
from databricks_distributed_deep_learning_amd.ops._native_gemm import force_kernel  # noqa: E402
from databricks_distributed_deep_learning_amd.ops.bridge import BNStats  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / it * 1000


dev = torch.device("cuda")
for cin, cout, k, s, H in [(64, 256, 1, 1, 56), (256, 64, 1, 1, 56), (64, 64, 3, 1, 56), (128, 128, 3, 1, 28),
                           (256, 1024, 1, 1, 14), (512, 512, 3, 1, 7), (512, 2048, 1, 1, 7)]:
    x = torch.randn(256, H, H, cin, device=dev).bfloat16()
    w = torch.randn(cout, k, k, cin, device=dev).bfloat16()
    row = []
    for kern in ("big", "small", "narrow"):
        with force_kernel(kern):
            a = t(lambda: NC._fwd(x, w, s, k // 2))
            b = t(lambda: NC._fwd(x, w, s, k // 2, stats=BNStats()))
        row.append(f"{kern} {a:7.1f}/{b:7.1f}us")
    print((cin, cout, k, s, H), "  ".join(row), flush=True)
