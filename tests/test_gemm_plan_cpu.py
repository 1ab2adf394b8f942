"""GEMM tuner candidate lists (ops/_native_gemm.py): pure host logic, no GPU.

* the "hybrid" row split is offered exactly when a 256x256-tile grid ends in a partial round and
  the remainder can be split-K over the chip (ViT-B/16: 297 / 891 tiles; not BERT-base's 192 /
  768-tile grids, which are under one round or whole rounds);
* its first launch covers whole rounds of tiles, so the split part is the partial round only;
* "big192" (256 x 192 tiles) is opt-in (DDL_GEMM_192=1) and only for N % 192 == 0.
"""
import importlib

import pytest

NG = importlib.import_module("databricks_distributed_deep_learning_amd.ops._native_gemm")


@pytest.mark.parametrize("M,N,K,expect", [
    (25216, 768, 768, (21760, 3)),      # ViT O-projection: 99 x 3 = 297 tiles
    (25216, 768, 3072, (21760, 6)),     # ViT FFN2: same grid, K = 3072 allows 6 splits
    (25216, 2304, 768, (21760, 2)),     # ViT QKV: 99 x 9 = 891 tiles, 126-tile remainder
    (16384, 768, 768, None),            # BERT: 192 tiles, under one round
    (16384, 3072, 768, None),           # BERT FFN1: 768 tiles, three whole rounds
    (25216, 3072, 768, None),           # ViT FFN1: 168-tile remainder cannot split within one round
    (25216, 768, 200, None),            # K not a whole number of 64-wide k-tiles
])
def test_hybrid_rows(M, N, K, expect):
    assert NG.hybrid_rows(M, N, K) == expect
    if expect is not None:
        m1, s = expect
        tn = -(-N // 256)
        assert m1 % 256 == 0 and (m1 // 256) * tn <= ((-(-M // 256) * tn) // NG.NUM_CU) * NG.NUM_CU
        assert (-(-(M - m1) // 256)) * tn * s <= NG.NUM_CU


def test_candidates_offer_hybrid_only_for_partial_rounds():
    kinds = {c[0] for c in NG._candidates(NG.MODE_NT, 25216, 768, 3072, False, 3072, 3072)}
    assert "hybrid" in kinds and "big" in kinds
    kinds = {c[0] for c in NG._candidates(NG.MODE_NT, 16384, 768, 3072, False, 3072, 3072)}
    assert "hybrid" not in kinds
    # weight-gradient (TN) and row-remapped GEMMs never take it
    assert not any(c[0] == "hybrid" for c in NG._candidates(NG.MODE_TN, 25216, 768, 3072, False, 768, 3072))
    assert not any(c[0] == "hybrid" for c in NG._candidates(NG.MODE_NT, 25216, 768, 3072, True, 3072, 3072))


def test_big192_is_opt_in(monkeypatch):
    assert not any(c[0] == "big192" for c in NG._candidates(NG.MODE_NT, 16384, 768, 768, False, 768, 768))
    monkeypatch.setattr(NG, "_BIG192", True)
    assert ("big192", 1) in NG._candidates(NG.MODE_NT, 16384, 768, 768, False, 768, 768)
    assert ("big192", 1) in NG._candidates(NG.MODE_NN, 16384, 2304, 768, False, 768, 2304)
    assert not any(c[0] == "big192" for c in NG._candidates(NG.MODE_NT, 16384, 1024, 768, False, 768, 768))


# ---- "blas" (hipBLASLt through torch.mm / addmm): which calls qualify, and the layout mapping ----
def _bf(*shape):
    import torch
    return torch.randn(*shape, dtype=torch.float32).to(torch.bfloat16)


def test_blas_ok_plain_calls_only():
    import torch
    C = torch.empty(4, 4, dtype=torch.bfloat16)
    b16, b32 = torch.zeros(4, dtype=torch.bfloat16), torch.zeros(4)
    ok = lambda mode=NG.MODE_NT, C=C, bias=None, act=None, aux=None, conv=None, rr=False, res=None, cs=None: \
        NG.blas_ok(mode, C, bias, act, aux, conv, rr, res, cs)  # noqa: E731
    assert ok() and ok(NG.MODE_NN) and ok(bias=b16) and ok(res=C)
    assert not ok(NG.MODE_TN) and not ok(NG.MODE_CONV)          # weight gradients / convolutions: native
    assert not ok(act="gelu") and not ok(act="dgelu", aux=C)     # fused epilogues: native
    assert not ok(bias=b32)                                      # fp32 bias on a bf16 GEMM
    assert not ok(bias=b16, res=C)                               # bias AND residual: one addmm input only
    assert not ok(cs=torch.empty(8)) and not ok(rr=True)
    assert not ok(C=torch.empty(4, 4))                           # fp32 output


@pytest.mark.parametrize("mode", ["NT", "NN"])
@pytest.mark.parametrize("epi", ["none", "bias", "residual", "residual_inplace", "accumulate"])
def test_blas_launch_matches_reference(mode, epi):
    """The "blas" launch reads the native operand layouts (row strides lda / ldb / ldc) and adds
    the same epilogue operands as the native kernels: checked against an fp32 reference on CPU."""
    import torch
    torch.manual_seed(0)
    M, N, K, ldc = 48, 40, 64, 56                     # ldc > N: a strided output block
    md = NG.MODE_NT if mode == "NT" else NG.MODE_NN
    A = _bf(M, K)
    B = _bf(N, K) if mode == "NT" else _bf(K, N)
    Bm = B.float().t() if mode == "NT" else B.float()
    C = _bf(M, ldc)
    C0 = C.clone()
    bias = _bf(N) if epi == "bias" else None
    res = None
    if epi == "residual":
        res = _bf(M, ldc)
    elif epi == "residual_inplace":
        res = C
    ref = A.float() @ Bm
    if bias is not None:
        ref = ref + bias.float()
    if res is not None:
        ref = ref + (C0 if res is C else res)[:, :N].float()
    if epi == "accumulate":
        ref = ref + C0[:, :N].float()
    NG._launch("blas", 1, md, A, K, B, B.shape[1], C, ldc, M, N, K, bias, None, None, None, False, res,
               epi == "accumulate")
    torch.testing.assert_close(C[:, :N].float(), ref, atol=0.1, rtol=0.02)
    assert torch.equal(C[:, N:], C0[:, N:])          # columns past N untouched
