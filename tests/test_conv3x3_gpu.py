"""Direct 3x3 convolution kernel (csrc/kernels/conv3x3.hip) against fp32 PyTorch.

Covers the forward (+ BatchNorm statistics rows), the BatchNorm-backward epilogue used
by the stride-1 dgrad, odd heights (a half-empty last row pair), W < 64 (masked pixel
slots), and workgroups that walk several row pairs / cross an image boundary (grid
smaller than the tile count: prefetched rows, ring-slot reuse, reload at image change)."""
from types import SimpleNamespace

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_conv(x, w):
    # x [N, H, W, C] bf16, w [K, 3, 3, C] bf16 -> fp32 [N, H, W, K]
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape,grid", [((2, 56, 56), 0), ((3, 7, 56), 0), ((2, 56, 56), 3), ((3, 9, 64), 2),
                                        ((1, 1, 56), 0)])
def test_direct3x3_forward_and_stats(shape, grid):
    from databricks_distributed_deep_learning_amd.ops import _native_conv as nc
    N, H, W = shape
    torch.manual_seed(0)
    x = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    w = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).bfloat16()
    y = torch.empty(N, H, W, 64, device="cuda", dtype=torch.bfloat16)
    part = torch.full((nc._direct3x3_rows(N * H * W) * 128,), float("nan"), device="cuda")
    rows = nc._direct3x3(x, w, y, part, grid=grid)
    torch.cuda.synchronize()
    ref = _ref_conv(x, w)
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    st = part[:rows * 128].view(rows, 2, 64).sum(0)
    yf = y.float().reshape(-1, 64)
    torch.testing.assert_close(st[0], yf.sum(0), atol=1e-1, rtol=1e-3)
    torch.testing.assert_close(st[1], (yf * yf).sum(0), atol=1e-1, rtol=1e-3)


@pytest.mark.parametrize("with_res,grid", [(False, 0), (True, 5)])
def test_direct3x3_bn_backward_epilogue(with_res, grid):
    from databricks_distributed_deep_learning_amd.ops import _native_conv as nc
    N, H, W = 2, 11, 56
    torch.manual_seed(1)
    dy = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    wt = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).bfloat16()
    aux = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    res = torch.randn(N, H, W, 64, device="cuda").bfloat16() if with_res else None
    mean = torch.randn(64, device="cuda") * 0.1
    istd = torch.rand(64, device="cuda") + 0.5
    bits = torch.rand(N * H * W * 64, device="cuda") > 0.3
    packed = (bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1)
    mask = packed.to(torch.uint8)
    hint = SimpleNamespace(x=aux, mask=mask, mean=mean, istd=istd)
    dx = torch.empty(N, H, W, 64, device="cuda", dtype=torch.bfloat16)
    part = torch.empty(nc._direct3x3_rows(N * H * W) * 128, device="cuda")
    rows = nc._direct3x3(dy, wt, dx, part, res=res, bnb=hint, grid=grid)
    torch.cuda.synchronize()
    v = _ref_conv(dy, wt)
    if res is not None:
        v = v + res.float()
    v = torch.where(bits.view(N, H, W, 64), v, torch.zeros_like(v))
    torch.testing.assert_close(dx.float(), v, atol=3e-2, rtol=2e-2)
    st = part[:rows * 128].view(rows, 2, 64).sum(0)
    d = dx.float().reshape(-1, 64)
    xhat = (aux.float().reshape(-1, 64) - mean) * istd
    torch.testing.assert_close(st[0], d.sum(0), atol=1e-1, rtol=1e-3)
    torch.testing.assert_close(st[1], (d * xhat).sum(0), atol=1e-1, rtol=1e-3)


def test_direct3x3_conv_autograd_matches_reference():
    """The autograd conv routes the 64->64 stride-1 3x3 through the direct kernel (fwd and dgrad)."""
    from databricks_distributed_deep_learning_amd.ops import _native_conv as nc
    torch.manual_seed(2)
    x = torch.randn(2, 56, 56, 64, device="cuda").bfloat16().requires_grad_()
    w = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).bfloat16().requires_grad_()
    assert nc._direct3x3_ok(x.shape, w.shape, 1, 1)
    y = nc.conv2d(x, w, 1, 1)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.detach().float().permute(0, 3, 1, 2).requires_grad_()
    yr = F.conv2d(xr, wr, padding=1)
    yr.backward(g.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(y.float(), yr.permute(0, 2, 3, 1), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad.permute(0, 2, 3, 1), atol=0.5, rtol=2e-2)


@pytest.mark.parametrize("shape,grid,acc,f32", [((2, 56, 56), 0, False, False), ((3, 7, 56), 2, True, False),
                                                 ((2, 9, 64), 3, False, True), ((1, 1, 56), 0, True, True)])
def test_direct3x3_wgrad(shape, grid, acc, f32):
    from databricks_distributed_deep_learning_amd.ops import _native_conv as nc
    N, H, W = shape
    torch.manual_seed(3)
    x = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    dy = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    xr = x.float().permute(0, 3, 1, 2)
    wr = torch.zeros(64, 64, 3, 3, device="cuda", requires_grad=True)
    F.conv2d(xr, wr, padding=1).backward(dy.float().permute(0, 3, 1, 2))
    ref = wr.grad.permute(0, 2, 3, 1)                       # [K, 3, 3, C]
    base = torch.randn(64, 3, 3, 64, device="cuda")
    dw = (base if f32 else base.bfloat16()).clone() if acc else \
        torch.empty(64, 3, 3, 64, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
    nc._direct3x3_wgrad(dy, x, dw, acc, grid=grid)
    torch.cuda.synchronize()
    want = ref + (base if f32 else base.bfloat16().float()) if acc else ref
    tol = dict(atol=0.05, rtol=1e-2) if f32 else dict(atol=0.25, rtol=1e-2)
    torch.testing.assert_close(dw.float(), want, **tol)
