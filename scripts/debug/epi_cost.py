"""Cost of the fused GEMM epilogues on BERT-base's FFN shapes (isolated, cache-cold, device time):
plain bf16 out vs + bias vs + bias + GELU (pre-activation stored) vs dGELU vs dGELU + bias-gradient
column sums vs + residual, all on the 256x256 kernel (``kernel="big"``) at the same tiling."""
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
    torch.cuda._sleep(int(3e5 * reps))
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


dev = torch.device("cuda")
T, H, F = 16384, 768, 3072
x = torch.randn(T, H, device=dev).bfloat16()
w1 = (torch.randn(F, H, device=dev) * 0.03).bfloat16()     # [out, in]
b1 = torch.randn(F, device=dev).bfloat16()
y = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
z = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
dh = torch.randn(T, H, device=dev).bfloat16()
w2 = (torch.randn(H, F, device=dev) * 0.03).bfloat16()     # FFN2 weight [H, F]
dz = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
part = torch.empty(G.stats_rows_max(T) * 2 * F, device=dev, dtype=torch.float32)
res = torch.randn(T, F, device=dev).bfloat16()
rows = []
for kind in ("big", "big192"):
    r = {}
    r["NT plain"] = t_us(lambda: G.gemm(G.MODE_NT, x, H, w1, H, y, F, T, F, H, kernel=kind))
    r["NT +bias"] = t_us(lambda: G.gemm(G.MODE_NT, x, H, w1, H, y, F, T, F, H, bias=b1, kernel=kind))
    r["NT +bias+gelu(+z)"] = t_us(lambda: G.gemm(G.MODE_NT, x, H, w1, H, y, F, T, F, H, bias=b1, act="gelu",
                                                 aux=z, kernel=kind))
    # dgrad of FFN2 into FFN1's output space: dZ = (dH W2) * GELU'(z), NN [T, H] x [H, F]
    r["NN plain"] = t_us(lambda: G.gemm(G.MODE_NN, dh, H, w2, F, dz, F, T, F, H, kernel=kind))
    r["NN +res"] = t_us(lambda: G.gemm(G.MODE_NN, dh, H, w2, F, dz, F, T, F, H, residual=res, kernel=kind))
    r["NN dgelu"] = t_us(lambda: G.gemm(G.MODE_NN, dh, H, w2, F, dz, F, T, F, H, act="dgelu", aux=z, kernel=kind))
    r["NN dgelu+colsums"] = t_us(lambda: G.gemm(G.MODE_NN, dh, H, w2, F, dz, F, T, F, H, act="dgelu", aux=z,
                                                colstats=part, kernel="big"))
    print(f"[{kind}] " + "  ".join(f"{k} {v:.1f}" for k, v in r.items()), flush=True)
