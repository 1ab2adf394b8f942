"""Precision of the bf16 split-K partial slabs of the weight-gradient GEMMs.

The TN weight-gradient kernels (``gemm_duo.hip`` TN, ``gemm_big.hip`` TN / ``gemm_wg_k``) store each
split's fp32 partial tile ROUNDED TO BF16, and the reduce sums those in fp32.  This test measures, on the
real BERT-base / ResNet-50 / BERT-large weight-gradient shapes at the split counts the committed plan
table runs (7-64 splits), the relative Frobenius error of that result against an fp64 reference -- next
to the unsplit kernel (one fp32 accumulation, ONE bf16 rounding: what an fp32-partial reduce would give up
to summation order) -- and pins it: the bf16 partials may add at most about ONE more bf16 rounding's
worth of error, in quadrature (S partials of size ~|sum| / sqrt(S), each rounded once: the added rms
error is sqrt(S) x r x |sum| / sqrt(S) = r x |sum| whatever S is; r = the rms relative error of one
bf16 rounding, 2^-7 / sqrt(12) x E[1 / mantissa] ~ 1.56e-3).  First measurement (round 6, 768 x 768 x
16384, 28 splits): unsplit 1.66e-3, split 2.35e-3 = sqrt(1.66^2 + 1.66^2) e-3.
"""
import json
import os

import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu

# (M = output features, N = input features, K = tokens / pixels, kernel, splits) -- ops/gemm_plans.json rows
CASES = [
    (768, 768, 16384, "duo", 28),       # BERT-base attention output / QKV blocks
    (3072, 768, 16384, "duo", 7),       # BERT-base FFN1
    (768, 3072, 16384, "duo", 7),       # BERT-base FFN2
    (2304, 768, 16384, "duo", 9),       # BERT-base QKV
    (256, 1024, 50176, "duo", 32),      # ResNet-50 stage-3 1x1
    (256, 512, 200704, "duo", 64),      # ResNet-50 stage-2 1x1
    (2048, 512, 12544, "duo", 8),       # ResNet-50 stage-4 1x1
    (1024, 4096, 16384, "big", 4),      # BERT-large FFN (256x256 TN)
    (768, 768, 16384, "wg", 8),         # 4-wave weight-gradient kernel
]


def _rel(x, ref):
    return ((x.double() - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("M,N,K,kind,splits", CASES)
def test_bf16_split_partials_error(M, N, K, kind, splits):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_TN, gemm
    torch.manual_seed(M * 7 + N + splits)
    # gradient-like operands: dz with ReLU-style zeros, activations of mixed scale
    dz = (torch.randn(K, M, device=dev) * (torch.rand(K, M, device=dev) > 0.5)).bfloat16()
    x = (torch.randn(K, N, device=dev) * (0.5 + torch.rand(1, N, device=dev))).bfloat16()
    ref = dz.double().t() @ x.double()
    out = {}
    for tag, kd, s in (("split", kind, splits), ("unsplit", "big", 1)):
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        gemm(MODE_TN, dz, M, x, N, c, N, M, N, K, kernel=kd, splits=s)
        torch.cuda.synchronize()
        out[tag] = _rel(c, ref)
    # accumulate form (into a bf16 gradient slot holding an earlier micro-step)
    prev = (torch.randn(M, N, device=dev) * ref.float().std()).bfloat16()
    acc = prev.clone()
    gemm(MODE_TN, dz, M, x, N, acc, N, M, N, K, kernel=kind, splits=splits, accumulate=True)
    out["accumulate"] = _rel(acc, ref + prev.double())
    rec = dict(M=M, N=N, K=K, kernel=kind, splits=splits, **{k: round(v, 7) for k, v in out.items()})
    print("splitk-precision", json.dumps(rec))
    log = os.environ.get("DDL_SPLITK_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(rec) + "\n")
    one_rounding = 2.0 ** -7 / 12 ** 0.5 * 0.6931   # rms relative error of one bf16 rounding (~1.56e-3)
    assert out["unsplit"] < 1.3 * one_rounding, out
    assert out["split"] ** 2 <= out["unsplit"] ** 2 + (1.25 * one_rounding) ** 2, out
    assert out["accumulate"] < 2.0 * one_rounding, out
