"""Streaming skinny GEMM (csrc/kernels/skinny_gemm.hip) against fp32 PyTorch: the ResNet
stage-1 1x1 conv shapes (N, K) = (256, 64) and (64, 256) with their epilogues -- BatchNorm
statistics rows, a residual, and the BatchNorm-backward reduction -- including an M that
is not a multiple of the 64-row tile and grids that give workgroups several tiles."""
import pytest
import torch

from databricks_distributed_deep_learning_amd.ops import _lib

pytestmark = pytest.mark.gpu


def _run(a, w, c, part=None, res=None, aux=None, mask=None, mean=None, istd=None, grid=0):
    M, K = a.shape
    N = w.shape[0]
    rc = _lib.fn("ddl_skinny_gemm")(a.data_ptr(), w.data_ptr(), c.data_ptr(), M, N, K, _lib.p(part), _lib.p(res),
                                    _lib.p(aux), _lib.p(mask), _lib.p(mean), _lib.p(istd), grid, _lib.stream())
    assert rc >= 0, rc
    torch.cuda.synchronize()
    return rc


@pytest.mark.parametrize("N,K", [(256, 64), (64, 256)])
@pytest.mark.parametrize("M,grid", [(4096, 0), (1000, 3), (64 * 37 + 5, 8)])
def test_skinny_plain_and_stats(N, K, M, grid):
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    part = torch.full((4096 * 2 * N,), float("nan"), device="cuda")
    rows = _run(a, w, c, part=part, grid=grid)
    ref = a.float() @ w.float().t()
    torch.testing.assert_close(c.float(), ref, atol=3e-2, rtol=2e-2)
    st = part[:rows * 2 * N].view(rows, 2, N).sum(0)
    cf = c.float()
    torch.testing.assert_close(st[0], cf.sum(0), atol=0.1, rtol=1e-3)
    torch.testing.assert_close(st[1], (cf * cf).sum(0), atol=0.1, rtol=1e-3)


@pytest.mark.parametrize("M,grid", [(4096, 0), (64 * 37 + 5, 8)])
def test_skinny_residual(M, grid):
    torch.manual_seed(1)
    a = torch.randn(M, 64, device="cuda").bfloat16()
    w = (torch.randn(256, 64, device="cuda") * 0.1).bfloat16()
    res = torch.randn(M, 256, device="cuda").bfloat16()
    c = torch.empty(M, 256, device="cuda", dtype=torch.bfloat16)
    _run(a, w, c, res=res, grid=grid)
    torch.testing.assert_close(c.float(), a.float() @ w.float().t() + res.float(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,grid,with_mask", [(4096, 0, True), (64 * 37 + 5, 8, True), (1000, 3, False)])
def test_skinny_bn_backward_epilogue(M, grid, with_mask):
    torch.manual_seed(2)
    a = torch.randn(M, 256, device="cuda").bfloat16()
    w = (torch.randn(64, 256, device="cuda") * 0.1).bfloat16()
    x = torch.randn(M, 64, device="cuda").bfloat16()
    mean = torch.randn(64, device="cuda") * 0.1
    istd = torch.rand(64, device="cuda") + 0.5
    bits = torch.rand(M * 64, device="cuda") > 0.3 if with_mask else torch.ones(M * 64, device="cuda", dtype=torch.bool)
    pad = (-bits.numel()) % 8
    bp = torch.cat([bits, torch.zeros(pad, dtype=torch.bool, device="cuda")])
    mask = (bp.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)
    c = torch.empty(M, 64, device="cuda", dtype=torch.bfloat16)
    part = torch.empty(4096 * 128, device="cuda")
    rows = _run(a, w, c, part=part, aux=x, mask=mask if with_mask else None, mean=mean, istd=istd, grid=grid)
    v = (a.float() @ w.float().t()) * bits.view(M, 64).float()
    torch.testing.assert_close(c.float(), v, atol=3e-2, rtol=2e-2)
    st = part[:rows * 128].view(rows, 2, 64).sum(0)
    d = c.float()
    xhat = (x.float() - mean) * istd
    torch.testing.assert_close(st[0], d.sum(0), atol=0.1, rtol=1e-3)
    torch.testing.assert_close(st[1], (d * xhat).sum(0), atol=0.1, rtol=1e-3)


@pytest.mark.parametrize("M,grid,with_mask", [(4096, 0, True), (64 * 37 + 5, 8, True), (64 * 9, 3, True),
                                              (1000, 5, False)])
def test_skinny_residual_bn_backward_epilogue(M, grid, with_mask):
    """N = 256 with residual AND the BatchNorm-backward epilogue (stage-1 residual dgrads):
    dz = (a w^T + res) * relu_mask, rows [sum dz | sum dz * xhat]; odd tile counts per
    workgroup exercise the two-tile unrolled loop's tail."""
    torch.manual_seed(3)
    N, K = 256, 64
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16()
    x = torch.randn(M, N, device="cuda").bfloat16()
    mean = torch.randn(N, device="cuda") * 0.1
    istd = torch.rand(N, device="cuda") + 0.5
    bits = torch.rand(M * N, device="cuda") > 0.3 if with_mask else torch.ones(M * N, device="cuda", dtype=torch.bool)
    mask = (bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    part = torch.full((4096 * 2 * N,), float("nan"), device="cuda")
    rows = _run(a, w, c, part=part, res=res, aux=x, mask=mask if with_mask else None, mean=mean, istd=istd, grid=grid)
    assert rows > 0
    v = (a.float() @ w.float().t() + res.float()) * bits.view(M, N).float()
    torch.testing.assert_close(c.float(), v, atol=3e-2, rtol=2e-2)
    st = part[:rows * 2 * N].view(rows, 2, N).sum(0)
    d = c.float()
    xhat = (x.float() - mean) * istd
    torch.testing.assert_close(st[0], d.sum(0), atol=0.1, rtol=1e-3)
    torch.testing.assert_close(st[1], (d * xhat).sum(0), atol=0.2, rtol=1e-3)
