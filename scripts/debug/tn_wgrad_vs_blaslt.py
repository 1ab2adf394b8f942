"""Time the BERT weight-gradient GEMMs (TN, K = tokens = 16384) on the native kernels
(tuned choice) against hipBLASLt via torch.addmm into the same bf16 gradient buffer."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_TN, gemm


def t_ms(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


dev = torch.device("cuda")
T = 16384
for N, K in [(768, 768), (2304, 768), (768, 3072), (3072, 768)]:
    dy = torch.randn(T, N, device=dev).bfloat16()
    x = torch.randn(T, K, device=dev).bfloat16()
    g = torch.zeros(N, K, device=dev).bfloat16()
    ours = t_ms(lambda: gemm(MODE_TN, dy, N, x, K, g, K, N, K, T, accumulate=True))
    g2 = torch.zeros(N, K, device=dev).bfloat16()
    lt = t_ms(lambda: torch.addmm(g2, dy.t(), x, out=g2))
    fl = 2.0 * T * N * K
    print(f"TN {N}x{K}x{T}: native {ours * 1e3:.1f} us ({fl / ours / 1e9:.0f} TF/s)  "
          f"hipBLASLt addmm {lt * 1e3:.1f} us ({fl / lt / 1e9:.0f} TF/s)", flush=True)

# forward (NT: y = x W^T) and input-gradient (NN: dx = dy W) shapes of BERT-base / ViT-B/16,
# plain epilogue, against torch.matmul (hipBLASLt) on the same operands
from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_NN, MODE_NT  # noqa: E402
for T in (16384, 25216):
    for N, K in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        x = torch.randn(T, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()
        y = torch.empty(T, N, device=dev).bfloat16()
        ours = t_ms(lambda: gemm(MODE_NT, x, K, w, K, y, N, T, N, K))
        lt = t_ms(lambda: torch.matmul(x, w.t(), out=y))
        dy = torch.randn(T, N, device=dev).bfloat16()
        dx = torch.empty(T, K, device=dev).bfloat16()
        ours2 = t_ms(lambda: gemm(MODE_NN, dy, N, w, K, dx, K, T, K, N))
        lt2 = t_ms(lambda: torch.matmul(dy, w, out=dx))
        fl = 2.0 * T * N * K
        print(f"T={T} NT {T}x{N}x{K}: native {ours * 1e3:.1f} us ({fl / ours / 1e9:.0f} TF/s)  hipBLASLt "
              f"{lt * 1e3:.1f} us ({fl / lt / 1e9:.0f} TF/s) | NN {T}x{K}x{N}: native {ours2 * 1e3:.1f} us "
              f"({fl / ours2 / 1e9:.0f})  hipBLASLt {lt2 * 1e3:.1f} us ({fl / lt2 / 1e9:.0f})", flush=True)
