"""Cost of the implicit-im2col B loader in the conv weight-gradient kernel (gemm_wg_k<true, 4>): the same
M x N x K weight gradient as CONVW (B = implicit im2col of the NHWC input) and as a plain TN GEMM over a
materialized im2col, both on kind "wg" at the plan's split count.  ResNet-50 stage-3 / stage-4 3x3 shapes."""
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


dev = torch.device("cuda")
for (Nb, H, C, K, splits) in [(256, 14, 256, 256, 14), (256, 7, 512, 512, 3)]:
    P = H
    M = Nb * P * P
    x = torch.randn(Nb, H, H, C, device=dev).bfloat16()
    dy = torch.randn(M, K, device=dev).bfloat16()
    dw = torch.zeros(K, 9 * C, device=dev).bfloat16()
    desc = _desc(Nb, H, H, C, P, P, 1, -1, -1, 1, 1, 3, 3, P, P)
    cols = torch.nn.functional.unfold(x.permute(0, 3, 1, 2).float(), 3, padding=1)       # [N, C*9, P*P]
    b = cols.view(Nb, C, 9, P * P).permute(0, 3, 2, 1).reshape(M, 9 * C).bfloat16().contiguous()
    fl = 2.0 * M * K * 9 * C
    cw = t_us(lambda: NG.gemm(NG.MODE_CONVW, dy, K, x, 0, dw, 9 * C, K, 9 * C, M, conv=desc, kernel="wg", splits=splits))
    tn = t_us(lambda: NG.gemm(NG.MODE_TN, dy, K, b, 9 * C, dw, 9 * C, K, 9 * C, M, kernel="wg", splits=splits))
    print(f"{K}x{9 * C}x{M} splits {splits}: CONVW {cw:.1f} us ({fl / cw / 1e6:.0f} TF)  TN over im2col {tn:.1f} us "
          f"({fl / tn / 1e6:.0f} TF)", flush=True)
