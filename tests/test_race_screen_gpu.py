"""Race screen: every deterministic kernel family is run repeatedly
on identical inputs and must reproduce its output BITWISE.

The GEMMs stage operands with asynchronous LDS-DMA under counted ``vmcnt`` and
staggered wave groups; a missing wait or a restage that overtakes a read shows
up as run-to-run differences long before it shows up as a tolerance failure.
Shapes cover odd K-tile counts (peeled last tile), K tails, split-K, all three
tile shapes and the implicit-GEMM conv loaders.  None of these kernels uses
atomics, so any difference is a race.
"""
import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu

REPS = 4


def _same(fn):
    outs = [fn().clone() for _ in range(REPS)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("kernel", ["big", "small", "narrow"])
@pytest.mark.parametrize("mode,M,N,K,splits", [(0, 1000, 2304, 832, None), (1, 4096, 768, 3072, None),
                                               (2, 768, 768, 8192, 4), (0, 2048, 2048, 4160, None),
                                               (0, 300, 520, 392, None)])
def test_gemm_bitwise_repeatable(kernel, mode, M, N, K, splits):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._native_gemm import gemm
    torch.manual_seed(0)
    if mode == 0:
        A, lda, B, ldb = torch.randn(M, K, device=dev).bfloat16(), K, torch.randn(N, K, device=dev).bfloat16(), K
    elif mode == 1:
        A, lda, B, ldb = torch.randn(M, K, device=dev).bfloat16(), K, torch.randn(K, N, device=dev).bfloat16(), N
    else:
        A, lda, B, ldb = torch.randn(K, M, device=dev).bfloat16(), M, torch.randn(K, N, device=dev).bfloat16(), N
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    _same(lambda: gemm(mode, A, lda, B, ldb, C, N, M, N, K, splits=splits, kernel=kernel))


@pytest.mark.parametrize("kernel", [None, "big", "small", "narrow"])
def test_conv_bitwise_repeatable(kernel):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    from databricks_distributed_deep_learning_amd.ops._native_gemm import force_kernel
    torch.manual_seed(1)
    x = torch.randn(8, 30, 30, 64, device=dev).bfloat16()
    w = torch.randn(128, 3, 3, 64, device=dev).bfloat16() * 0.05
    dy = torch.randn(8, 15, 15, 128, device=dev).bfloat16()
    with force_kernel(kernel):
        _same(lambda: NC._fwd(x, w, 2, 1))
        _same(lambda: NC._dgrad(dy, w, x.shape, 2, 1))
        _same(lambda: NC._wgrad(dy, x, w.shape, 2, 1))


def test_attention_bn_ln_bitwise_repeatable():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(2)
    qkv = torch.randn(4, 197, 3 * 768, device=dev).bfloat16()
    mask = torch.ones(4, 197, device=dev)
    _same(lambda: ops.attention(qkv, 12, mask))
    x = torch.randn(4096, 256, device=dev).bfloat16()
    g = torch.ones(256, device=dev).bfloat16()
    b = torch.zeros(256, device=dev).bfloat16()
    _same(lambda: ops.layer_norm(x, g, b, 1e-12))
    xb = torch.randn(8, 28, 28, 256, device=dev).bfloat16()
    rm, rv = torch.zeros(256, device=dev), torch.ones(256, device=dev)
    _same(lambda: ops.batch_norm(xb, g, b, rm.clone(), rv.clone(), True, 0.1, 1e-5, True, None))


def test_embedding_backward_bitwise_repeatable():
    """Word-embedding gradient with heavily repeated ids (padding, [CLS]-like tokens): the sorted
    segmented sum has no atomics, so the gradient is the same bits every run."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_embedding as Em
    torch.manual_seed(3)
    w = torch.randn(30522, 768, device=dev).bfloat16()
    ids = torch.randint(0, 30522, (64, 128), device=dev)
    ids[:, 0] = 101
    ids[:, 90:] = 0
    g = torch.randn(64, 128, 768, device=dev).bfloat16()

    def run():
        ww = w.clone().requires_grad_(True)
        Em.embedding(ids, ww).backward(g)
        return ww.grad

    _same(run)
