"""Register-B streaming GEMM (csrc/kernels/stream_gemm.hip) against fp32 PyTorch: the ResNet
stage-2 1x1 conv shapes (N, K) = (512, 128) and (128, 512) with their epilogues -- BatchNorm
statistics rows (forward), the BatchNorm-backward reduction (dgrad) and that plus the
block-input residual -- including an M that is not a multiple of the tile, odd tile counts per
workgroup (the two-tile unrolled loop's tail) and grids that give workgroups many tiles."""
import pytest
import torch

from databricks_distributed_deep_learning_amd.ops import _lib

pytestmark = pytest.mark.gpu


def _run(a, w, c, part=None, res=None, aux=None, mask=None, mean=None, istd=None, grid=0):
    M, K = a.shape
    N = w.shape[0]
    rc = _lib.fn("ddl_stream_gemm")(a.data_ptr(), w.data_ptr(), c.data_ptr(), M, N, K, _lib.p(part), _lib.p(res),
                                    _lib.p(aux), _lib.p(mask), _lib.p(mean), _lib.p(istd), grid, _lib.stream())
    assert rc >= 0, rc
    torch.cuda.synchronize()
    return rc


def _mask(bits):
    return (bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)


@pytest.mark.parametrize("N,K", [(512, 128), (128, 512), (1024, 256), (256, 1024)])
@pytest.mark.parametrize("M,grid", [(8192, 0), (1000, 3), (64 * 37 + 5, 8), (200704, 0), (50176, 0)])
def test_stream_plain_and_stats(N, K, M, grid):
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    part = torch.full((256 * 2 * N,), float("nan"), device="cuda")
    rows = _run(a, w, c, part=part, grid=grid)
    ref = a.float() @ w.float().t()
    torch.testing.assert_close(c.float(), ref, atol=5e-2, rtol=2e-2)
    st = part[:rows * 2 * N].view(rows, 2, N).sum(0)
    cf = c.float()
    torch.testing.assert_close(st[0], cf.sum(0), atol=0.5, rtol=1e-3)
    torch.testing.assert_close(st[1], (cf * cf).sum(0), atol=0.5, rtol=1e-3)


@pytest.mark.parametrize("N,K", [(512, 128), (128, 512), (1024, 256), (256, 1024)])
@pytest.mark.parametrize("M,grid,with_mask,with_res", [(8192, 0, True, True), (32 * 37 + 5, 8, True, True),
                                                       (32 * 9, 3, True, False), (1000, 5, False, True),
                                                       (50000, 0, True, False)])
def test_stream_bn_backward_epilogue(N, K, M, grid, with_mask, with_res):
    """dz = (a w^T [+ res]) * relu_mask, rows [sum dz | sum dz * xhat] (residual: N = 512 only)."""
    if with_res and N not in (512, 1024):
        pytest.skip("residual epilogue: N = 512 / 1024 (the residual-adding stage-2 / 3 dgrads)")
    torch.manual_seed(3)
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16() if with_res else None
    x = torch.randn(M, N, device="cuda").bfloat16()
    mean = torch.randn(N, device="cuda") * 0.1
    istd = torch.rand(N, device="cuda") + 0.5
    bits = torch.rand(M * N, device="cuda") > 0.3 if with_mask else torch.ones(M * N, device="cuda", dtype=torch.bool)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    part = torch.full((256 * 2 * N,), float("nan"), device="cuda")
    rows = _run(a, w, c, part=part, res=res, aux=x, mask=_mask(bits) if with_mask else None, mean=mean, istd=istd,
                grid=grid)
    assert rows > 0
    v = a.float() @ w.float().t()
    if res is not None:
        v = v + res.float()
    v = v * bits.view(M, N).float()
    torch.testing.assert_close(c.float(), v, atol=5e-2, rtol=2e-2)
    st = part[:rows * 2 * N].view(rows, 2, N).sum(0)
    d = c.float()
    xhat = (x.float() - mean) * istd
    torch.testing.assert_close(st[0], d.sum(0), atol=0.5, rtol=1e-3)
    torch.testing.assert_close(st[1], (d * xhat).sum(0), atol=0.5, rtol=1e-3)


def test_stream_not_covered():
    a = torch.randn(64, 256, device="cuda").bfloat16()
    w = torch.randn(64, 256, device="cuda").bfloat16()
    c = torch.empty(64, 64, device="cuda", dtype=torch.bfloat16)
    rc = _lib.fn("ddl_stream_gemm")(a.data_ptr(), w.data_ptr(), c.data_ptr(), 64, 64, 256, 0, 0, 0, 0, 0, 0, 0,
                                    _lib.stream())
    assert rc == -1


@pytest.mark.parametrize("M,N", [(256, 64), (64, 256), (64, 64), (512, 128), (128, 512), (128, 256), (256, 256)])
@pytest.mark.parametrize("K,accumulate", [(200704, False), (50000 + 17, True)])
def test_stream_wgrad(M, N, K, accumulate):
    """Streaming weight gradient C (+)= A^T B (A = [K][M] output gradient, B = [K][N] input) on the
    register-accumulator kernel ("swg": whole M x N output per workgroup, bf16 partials + reduce),
    against fp32; K not a multiple of the 32-row slot (the zero-page tail)."""
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(7)
    a = torch.randn(K, M, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16()
    c0 = (torch.randn(M, N, device="cuda") * 100).bfloat16()
    c = c0.clone()
    NG.gemm(NG.MODE_TN, a, M, b, N, c, N, M, N, K, accumulate=accumulate, kernel="swg")
    torch.cuda.synchronize()
    ref = a.float().t() @ b.float() + (c0.float() if accumulate else 0)
    err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-2, err
