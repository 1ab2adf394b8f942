"""Cross-kernel fusions on the GPU: BatchNorm statistics produced by the conv GEMM
epilogue (``gemm(colstats=...)`` -> ``ddl_bn_fwd_from_partials``) must match the
standalone statistics pass, for every tile variant and odd M / N tails."""
import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel", ["big", "small", "narrow"])
@pytest.mark.parametrize("N,H,C,K,R,stride", [(4, 20, 64, 64, 3, 1), (2, 17, 32, 256, 1, 1), (3, 15, 64, 256, 3, 2),
                                              (8, 28, 128, 512, 1, 1), (32, 56, 64, 256, 1, 1),
                                              (16, 30, 64, 128, 3, 1)])
def test_bn_stats_from_gemm_epilogue(kernel, N, H, C, K, R, stride):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.ops._native_gemm import force_kernel
    from databricks_distributed_deep_learning_amd.ops.bridge import BNStats
    torch.manual_seed(3)
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    w = (torch.randn(K, R, R, C, device=dev) * 0.1).bfloat16()
    g = (torch.rand(K, device=dev) + 0.5).bfloat16()
    b = torch.randn(K, device=dev).bfloat16()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    NC.STATS_MIN_K, saved = 0, NC.STATS_MIN_K        # exercise the epilogue on every shape
    try:
        outs = _run(x, w, g, b, K, R, stride, kernel, force_kernel, BNStats, ops, dev)
    finally:
        NC.STATS_MIN_K = saved
    (z0, m0, v0), (z1, m1, v1) = outs
    torch.testing.assert_close(m1, m0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(v1, v0, rtol=1e-3, atol=1e-5)
    assert ((z1 - z0).abs().max() / z0.abs().max()).item() < 1e-2


def _run(x, w, g, b, K, R, stride, kernel, force_kernel, BNStats, ops, dev):
    outs = []
    for fused in (False, True):
        rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
        st = BNStats() if fused else None
        with force_kernel(kernel):
            y = ops.conv2d(x, w, stride, R // 2, bn_stats=st)
        if fused:
            assert st.part is not None, "GEMM epilogue produced no statistics"
        z = ops.batch_norm(y, g, b, rm, rv, True, 0.1, 1e-5, True, None, stats=st)
        if fused:
            assert st.part is None, "BN did not consume the epilogue statistics"
        outs.append((z.float(), rm, rv))
    return outs
