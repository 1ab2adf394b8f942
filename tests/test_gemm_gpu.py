"""MFMA GEMM / implicit-GEMM conv numerics vs fp32 PyTorch references (GPU only).

Asymmetric random operands throughout (a transposed C-write cannot pass), odd
shapes that exercise every M/N/K tail path, and every loader layout.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import gpu_device

pytestmark = pytest.mark.gpu


def _rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


SHAPES = [(128, 128, 64), (256, 384, 768), (77, 200, 136), (1000, 2304, 768), (130, 8, 72), (16, 1000, 2048)]


@pytest.mark.parametrize("kernel", ["big", "small", "narrow"])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_modes(M, N, K, kernel):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_NN, MODE_NT, MODE_TN, force_kernel
    from databricks_distributed_deep_learning_amd.ops._native_gemm import gemm as _gemm

    def gemm(*a, **k):
        with force_kernel(kernel):
            return _gemm(*a, **k)
    torch.manual_seed(0)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    ref = a.float() @ w.float().t()
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    gemm(MODE_NT, a, K, w, K, c, N, M, N, K)
    assert _rel_err(c, ref) < 1e-2
    # NN: dx = dy @ W  (dy [M, N], W [N, K])
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    gemm(MODE_NN, dy, N, w, K, dx, K, M, K, N)
    assert _rel_err(dx, dy.float() @ w.float()) < 1e-2
    # TN: dW = dy^T @ a  -> [N, K], reduction over M (split-K path for small tiles)
    dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    gemm(MODE_TN, dy, N, a, K, dw, K, N, K, M)
    assert _rel_err(dw, dy.float().t() @ a.float()) < 1e-2
    dw32 = torch.empty(N, K, device=dev, dtype=torch.float32)
    gemm(MODE_TN, dy, N, a, K, dw32, K, N, K, M, splits=3)
    assert _rel_err(dw32, dy.float().t() @ a.float()) < 1e-3


@pytest.mark.parametrize("kind", ["wg", "wg2"])
@pytest.mark.parametrize("Mo,No,Kr", [(256, 256, 128), (512, 512, 1152), (768, 256, 4096), (2304, 768, 1024),
                                      (512, 384, 512)])
@pytest.mark.parametrize("splits", [1, 2, 5])
def test_wgrad_kernel(Mo, No, Kr, splits, kind):
    """4-wave weight-gradient kernel ("wg", gemm_big.hip gemm_wg_k): dW = dY^T X over the reduction,
    fp32 partials + reduce; bf16 / fp32 outputs, plain and accumulating, vs an fp32 reference."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_TN, gemm
    torch.manual_seed(Mo + No + Kr + splits)
    dy = torch.randn(Kr, Mo, device=dev).to(torch.bfloat16)
    x = torch.randn(Kr, No, device=dev).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    dw = torch.empty(Mo, No, device=dev, dtype=torch.bfloat16)
    gemm(MODE_TN, dy, Mo, x, No, dw, No, Mo, No, Kr, kernel=kind, splits=splits)
    assert _rel_err(dw, ref) < 1e-2
    prev = torch.randn(Mo, No, device=dev)
    acc32 = prev.clone()
    gemm(MODE_TN, dy, Mo, x, No, acc32, No, Mo, No, Kr, kernel=kind, splits=splits, accumulate=True)
    assert _rel_err(acc32, prev + ref) < 1e-3
    acc16 = prev.to(torch.bfloat16)
    gemm(MODE_TN, dy, Mo, x, No, acc16, No, Mo, No, Kr, kernel=kind, splits=splits, accumulate=True)
    assert _rel_err(acc16, prev + ref) < 1e-2


def test_wgrad_kernel_contract():
    """Shapes outside the 4-wave kernel's contract (M % 256, N % 128, K % 128) run another kernel."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    assert NG.wg_ok(768, 2304, 16384, 768, 2304) and not NG.wg_ok(200, 256, 64, 200, 256)
    assert not NG.wg_ok(256, 256, 48, 256, 256) and not NG.wg_ok(256, 256, 96, 256, 256)
    dy = torch.randn(96, 200, device=dev).to(torch.bfloat16)
    x = torch.randn(96, 256, device=dev).to(torch.bfloat16)
    dw = torch.empty(200, 256, device=dev, dtype=torch.bfloat16)
    NG.gemm(NG.MODE_TN, dy, 200, x, 256, dw, 256, 200, 256, 96, kernel="wg")
    assert _rel_err(dw, dy.float().t() @ x.float()) < 1e-2


@pytest.mark.parametrize("act", [None, "gelu", "relu", "tanh"])
def test_linear_autograd(act):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_linear
    from databricks_distributed_deep_learning_amd.ops.linear import linear_reference
    torch.manual_seed(1)
    x = torch.randn(3, 50, 96, device=dev).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(136, 96, device=dev) * 0.1).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(136, device=dev).to(torch.bfloat16).requires_grad_(True)
    y = _native_linear.linear(x, w, b, act)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = linear_reference(xr, wr, br, act)
    assert _rel_err(y, yr) < 2e-2
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    for got, want in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert _rel_err(got, want) < 3e-2


@pytest.mark.parametrize("N,act", [(2, None), (5, "tanh"), (1000 + 3, None)])
def test_linear_padded_n_native(N, act, monkeypatch):
    """N % 8 != 0 (BERT's classifier head, num_labels = 2) runs on the native GEMMs over N padded
    to 8 (no hipBLASLt): forward and all three gradients against fp32 autograd."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_linear
    from databricks_distributed_deep_learning_amd.ops.linear import linear_reference
    called = []
    orig = torch.nn.functional.linear

    def spy(*a, **k):      # F.linear on GPU tensors = hipBLASLt
        called.append(1)
        return orig(*a, **k)
    monkeypatch.setattr(torch.nn.functional, "linear", spy)
    torch.manual_seed(2)
    x = torch.randn(128, 768, device=dev).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(N, 768, device=dev) * 0.05).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(N, device=dev).to(torch.bfloat16).requires_grad_(True)
    y = _native_linear.linear(x, w, b, act)
    g = torch.randn(128, N, device=dev)
    y.backward(g.to(torch.bfloat16))
    assert not called and y.shape == (128, N)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = linear_reference(xr, wr, br, act)
    assert _rel_err(y, yr) < 2e-2
    yr.backward(g.to(torch.bfloat16).float())
    for got, want in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert got.shape == want.shape and _rel_err(got, want) < 3e-2


CONVS = [  # N, H, W, C, K, R, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 15, 13, 64, 128, 3, 2, 1),
    (2, 16, 16, 256, 512, 1, 2, 0),
    (2, 9, 11, 128, 64, 1, 1, 0),
    (2, 32, 30, 3, 64, 7, 2, 3),
    (1, 7, 7, 512, 512, 3, 1, 1),
    (8, 56, 56, 64, 256, 3, 1, 1),      # large-tile CONV fwd + CONVW wgrad
    (8, 28, 28, 256, 512, 1, 1, 0),     # large-tile NT / NN / TN
    (8, 30, 30, 256, 256, 3, 2, 1),     # stride-2 parity classes
]


@pytest.mark.parametrize("kernel", [None, "big", "small", "narrow", "duo"])
@pytest.mark.parametrize("N,H,W,C,K,R,stride,pad", CONVS)
def test_conv_fwd_bwd(N, H, W, C, K, R, stride, pad, kernel):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv
    from databricks_distributed_deep_learning_amd.ops._native_gemm import force_kernel
    with force_kernel(kernel):
        _conv_case(dev, N, H, W, C, K, R, stride, pad)


def _conv_case(dev, N, H, W, C, K, R, stride, pad):
    from databricks_distributed_deep_learning_amd.ops import _native_conv
    from databricks_distributed_deep_learning_amd.ops.conv import conv2d_reference
    torch.manual_seed(2)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(K, R, R, C, device=dev) / (R * (C ** 0.5))).to(torch.bfloat16).requires_grad_(True)
    y = _native_conv.conv2d(x, w, stride, pad)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = conv2d_reference(xr, wr, stride, pad)
    assert y.shape == yr.shape
    assert _rel_err(y, yr) < 2e-2
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    assert _rel_err(x.grad, xr.grad) < 2e-2
    assert _rel_err(w.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (4096, 2304, 768), (1000, 3000, 264), (2048, 768, 3072),
                                   (300, 520, 392)])
def test_big_gemm_modes(mode, M, N, K):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(4)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    if mode == 0:      # C[M,N] = a w^T + b, gelu (aux = pre-activation)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        z = torch.empty_like(c)
        NG.gemm(0, a, K, w, K, c, N, M, N, K, bias=b, act="gelu", aux=z, kernel="big")
        pre = a.float() @ w.float().t() + b.float()
        assert _rel_err(c, torch.nn.functional.gelu(pre)) < 1e-2 and _rel_err(z, pre) < 1e-2
    elif mode == 1:    # dx[M,K] = dy[M,N] w[N,K]
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        NG.gemm(1, dy, N, w, K, dx, K, M, K, N, kernel="big")
        assert _rel_err(dx, dy.float() @ w.float()) < 1e-2
    else:              # dW[N,K] (+)= dy^T a, split-K; accumulate into an existing grad
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        dw = torch.randn(N, K, device=dev).to(torch.bfloat16)
        base = dw.float().clone()
        NG.gemm(2, dy, N, a, K, dw, K, N, K, M, accumulate=True, kernel="big")
        assert _rel_err(dw, base + dy.float().t() @ a.float()) < 1e-2


@pytest.mark.parametrize("splits", [None, 1, 3])
@pytest.mark.parametrize("M,N,K", [(64, 576, 3000), (64, 256, 4096), (128, 1152, 777 * 8), (40, 72, 520)])
def test_transposed_weight_gradient(M, N, K, splits):
    """dW computed as (x^T dy)^T with the 64-channel side on the 128x64 tile's N extent
    (kernel "tnarrow": operands swapped, C^T stored, accumulate into an existing grad)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(7)
    dy = torch.randn(K, M, device=dev).to(torch.bfloat16)     # [pixels, Cout]
    x = torch.randn(K, N, device=dev).to(torch.bfloat16)      # [pixels, Cin]
    base = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dw = base.clone()
    NG.gemm(NG.MODE_TN, dy, M, x, N, dw, N, M, N, K, accumulate=True, kernel="tnarrow", splits=splits)
    assert _rel_err(dw, base.float() + dy.float().t() @ x.float()) < 1e-2


@pytest.mark.parametrize("N,H,W,C,K,R,stride,pad", [(4, 20, 20, 64, 64, 3, 1, 1), (2, 30, 30, 8, 64, 7, 2, 3),
                                                    (4, 14, 14, 128, 64, 3, 2, 1)])
def test_conv_wgrad_transposed(N, H, W, C, K, R, stride, pad):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    from databricks_distributed_deep_learning_amd.ops._native_gemm import force_kernel
    from databricks_distributed_deep_learning_amd.ops.conv import conv2d_reference
    torch.manual_seed(8)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(K, R, R, C, device=dev).to(torch.bfloat16)
    P = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, P, P, K, device=dev).to(torch.bfloat16)
    xr = x.float().requires_grad_(False)
    wr = w.float().requires_grad_(True)
    conv2d_reference(xr, wr, stride, pad).backward(dy.float())
    with force_kernel("tnarrow"):
        dw = NC._wgrad(dy, x, w.shape, stride, pad)
    assert _rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("N,H,W,C,K,R,stride,pad", [(2, 16, 16, 128, 256, 3, 1, 1), (2, 32, 32, 128, 256, 3, 2, 1),
                                                    (2, 16, 16, 256, 512, 3, 2, 1)])
@pytest.mark.parametrize("kind", ["wg", "wg2"])
def test_conv_wgrad_wg(N, H, W, C, K, R, stride, pad, kind):
    """Conv weight gradient on the 4-wave kernel with an implicit-im2col B operand ("wg", CONVW):
    padding taps from the zero page, stride 2, vs the fp32 reference."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    from databricks_distributed_deep_learning_amd.ops.conv import conv2d_reference
    torch.manual_seed(10)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(K, R, R, C, device=dev).to(torch.bfloat16)
    P = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, P, P, K, device=dev).to(torch.bfloat16)
    assert NG.wg_ok(K, R * R * C, N * P * P, K, 0)
    wr = w.float().requires_grad_(True)
    conv2d_reference(x.float(), wr, stride, pad).backward(dy.float())
    with NG.force_kernel(kind):
        dw = NC._wgrad(dy, x, w.shape, stride, pad)
    assert _rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("path", ["serial", "multi", "multi_narrow"])
@pytest.mark.parametrize("N,H,W,C,K,R,pad", [(2, 15, 13, 64, 128, 3, 1), (4, 28, 28, 128, 128, 3, 1),
                                             (2, 9, 9, 64, 64, 5, 2)])
def test_strided_dgrad_class_paths(path, N, H, W, C, K, R, pad):
    """Stride-2 dgrad: per-class launches vs the single multi-class launch (ddl_gemm_conv_multi)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    from databricks_distributed_deep_learning_amd.ops.conv import conv2d_reference
    torch.manual_seed(9)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=dev) / (R * C ** 0.5)).to(torch.bfloat16)
    P = (H + 2 * pad - R) // 2 + 1
    Q = (W + 2 * pad - R) // 2 + 1
    dy = torch.randn(N, P, Q, K, device=dev).to(torch.bfloat16)
    key = (tuple(dy.shape), tuple(w.shape), 2, pad)
    NC._MULTI_CHOICE[key] = path
    try:
        dx = NC._dgrad(dy, w, x.shape, 2, pad)
    finally:
        NC._MULTI_CHOICE.pop(key, None)
    xr = x.float().requires_grad_(True)
    conv2d_reference(xr, w.float(), 2, pad).backward(dy.float())
    assert _rel_err(dx, xr.grad) < 2e-2


@pytest.mark.parametrize("M,N,K", [(8292, 2304, 136), (4100, 4200, 768), (520, 264, 1024), (70000, 512, 64),
                                   (70000, 256, 128)])
@pytest.mark.parametrize("variant", ["plain", "bias_bf16_relu", "bias_f32", "acc_f32", "acc_bf16", "residual",
                                     "bias_gelu_aux"])
def test_big_direct_persistent_epilogue(M, N, K, variant):
    """Register epilogue + persistent grid of the 256x256 kernel (> 256 tiles: blocks
    walk several tiles, the next tile's prologue overlaps this tile's stores)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(7)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    ref = a.float() @ w.float().t()
    kw = {}
    out_dtype = torch.bfloat16
    if variant == "bias_bf16_relu":
        b = torch.randn(N, device=dev).to(torch.bfloat16)
        kw = dict(bias=b, act="relu")
        ref = torch.relu(ref + b.float())
    elif variant == "bias_f32":
        b = torch.randn(N, device=dev)
        kw = dict(bias=b)
        ref = ref + b
    elif variant.startswith("acc"):
        out_dtype = torch.float32 if variant == "acc_f32" else torch.bfloat16
        kw = dict(accumulate=True)
    elif variant == "residual":
        r = torch.randn(M, N, device=dev).to(torch.bfloat16)
        kw = dict(residual=r)
        ref = ref + r.float()
    elif variant == "bias_gelu_aux":
        b = torch.randn(N, device=dev).to(torch.bfloat16)
        z = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        kw = dict(bias=b, act="gelu", aux=z)
        pre = ref + b.float()
        ref = torch.nn.functional.gelu(pre)
    c = torch.randn(M, N, device=dev).to(out_dtype)
    if variant.startswith("acc"):
        ref = ref + c.float()
    NG.gemm(0, a, K, w, K, c, N, M, N, K, kernel="big", **kw)
    assert _rel_err(c, ref) < (2e-3 if out_dtype == torch.float32 else 1e-2)
    if variant == "bias_gelu_aux":
        assert _rel_err(z, pre) < 1e-2
    # every output element written exactly once: a second run into a NaN-filled
    # buffer must leave no NaN (non-accumulating variants)
    if not variant.startswith("acc"):
        c2 = torch.full((M, N), float("nan"), device=dev, dtype=out_dtype)
        NG.gemm(0, a, K, w, K, c2, N, M, N, K, kernel="big", **kw)
        assert not torch.isnan(c2).any()
        assert torch.equal(c2, c)


@pytest.mark.parametrize("M", [4096, 1000])
def test_ffn_dgelu_handoff(M):
    """FFN: Linear(gelu) -> Linear(fuse_dgelu=True).  The second layer's dgrad epilogue
    applies the first layer's dGELU and column-sums its bias gradient; every gradient
    must match an fp32 reference (M=1000 leaves edge tiles on the general path)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(12)
    H, I = 768, 3072
    x = torch.randn(M, H, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(I, H, device=dev) / H ** 0.5).to(torch.bfloat16)
    b1 = (torch.randn(I, device=dev) * 0.1).to(torch.bfloat16)
    w2 = (torch.randn(H, I, device=dev) / I ** 0.5).to(torch.bfloat16)
    b2 = (torch.randn(H, device=dev) * 0.1).to(torch.bfloat16)
    a = [t.clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    f = [t.float().clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    y = ops.linear(ops.linear(a[0], a[1], a[2], "gelu"), a[3], a[4], None, fuse_dgelu=True)
    yr = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(f[0], f[1], f[2])), f[3], f[4])
    assert _rel_err(y, yr) < 2e-2
    dy = torch.randn(M, H, device=dev)
    y.backward(dy.to(torch.bfloat16))
    yr.backward(dy)
    for t, r, name in zip(a, f, ("dx", "dw1", "db1", "dw2", "db2")):
        assert _rel_err(t.grad, r.grad) < 3e-2, name


@pytest.mark.parametrize("H,W", [(224, 224), (57, 61), (128, 96)])
def test_stem_space_to_depth(H, W):
    """7x7/2 RGB stem through the space-to-depth path: forward and weight gradient
    against fp32 F.conv2d (odd extents exercise the padded block row / column)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(13)
    x = torch.randn(4, H, W, 3, device=dev).to(torch.bfloat16)
    w = (torch.randn(64, 7, 7, 3, device=dev) * 0.1).to(torch.bfloat16).requires_grad_(True)
    y = ops.conv2d(x, w, 2, 3)
    wr = w.detach().float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    yr = F.conv2d(x.float().permute(0, 3, 1, 2), wr, stride=2, padding=3).permute(0, 2, 3, 1)
    assert y.shape == yr.shape
    assert _rel_err(y, yr) < 1e-2
    dy = torch.randn_like(yr)
    y.backward(dy.to(torch.bfloat16))
    yr.backward(dy)
    assert _rel_err(w.grad, wr.grad.permute(0, 2, 3, 1)) < 2e-2


@pytest.mark.parametrize("N,P,Q,grid", [(2, 8, 112, 0), (3, 12, 64, 5), (1, 4, 16, 0), (2, 112, 112, 7),
                                        (1, 8, 48, 0)])
@pytest.mark.parametrize("with_stats", [False, True])
def test_stem_fwd_kernel(N, P, Q, grid, with_stats):
    """Direct stem forward (stem_conv.hip) on space-to-depth operands against fp32 F.conv2d,
    and its BatchNorm partial sums against the sums of the stored bf16 output."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    torch.manual_seed(P + Q + N)
    xs = torch.randn(N, P + 3, Q + 3, 16, device=dev).to(torch.bfloat16)
    ws = (torch.randn(64, 4, 4, 16, device=dev) * 0.1).to(torch.bfloat16)
    assert NC._stem_fwd_ok(xs, ws)

    class Rec:
        def set(self, y, part, rows):
            self.part, self.rows = part, rows
    rec = Rec() if with_stats else None
    y = NC._stem_fwd(xs, ws, rec, grid=grid)
    ref = F.conv2d(xs.float().permute(0, 3, 1, 2), ws.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert _rel_err(y, ref) < 1e-2
    if with_stats:
        part = rec.part[:rec.rows * 128].view(rec.rows, 2, 64).sum(0)
        yf = y.float().reshape(-1, 64)
        torch.testing.assert_close(part[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.shape[0] ** 0.5)
        torch.testing.assert_close(part[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("N,P,Q,grid", [(2, 8, 112, 0), (3, 6, 64, 4), (1, 4, 16, 0), (2, 112, 112, 7)])
@pytest.mark.parametrize("out_dtype,accumulate", [(torch.bfloat16, False), (torch.float32, True)])
def test_stem_wgrad_kernel(N, P, Q, grid, out_dtype, accumulate):
    """Direct stem weight gradient (stem_wgrad.hip) on space-to-depth operands against the fp32
    tap-by-tap reference, written in the original [64, 7, 7, 3] layout; grids that split the
    row pairs unevenly, several row widths (tile templates), accumulate into an fp32 sink."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    torch.manual_seed(P * Q + N)
    xs = torch.randn(N, P + 3, Q + 3, 16, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, P, Q, 64, device=dev).to(torch.bfloat16)
    assert NC._stem_wgrad_ok(xs, dy, (64, 4, 4, 16), (64, 7, 7, 3))
    ref = torch.empty(64, 4, 4, 16, device=dev)
    xf, df = xs.float(), dy.float()
    for r in range(4):
        for s in range(4):
            ref[:, r, s] = torch.einsum("npqk,npqc->kc", df, xf[:, r:r + P, s:s + Q])
    ref = NC._s2d_weight_grad(ref, (64, 7, 7, 3))
    base = torch.randn(64, 7, 7, 3, device=dev).to(out_dtype) if accumulate else None
    dw = base.clone() if accumulate else torch.empty(64, 7, 7, 3, device=dev, dtype=out_dtype)
    NC._stem_wgrad(xs, dy, dw, accumulate, grid=grid)
    torch.cuda.synchronize()
    want = ref + base.float() if accumulate else ref
    assert _rel_err(dw, want) < 1e-2


@pytest.mark.parametrize("splits", [8, 32, 64])
@pytest.mark.parametrize("kernel", ["small", "narrow", "tnarrow"])
@pytest.mark.parametrize("accumulate,with_bias,out_f32", [(False, False, False), (True, False, True),
                                                          (False, True, True), (True, True, False)])
def test_split_k_reduce_thread_groups(splits, kernel, accumulate, with_bias, out_f32):
    """Weight-gradient GEMMs with 8 / 32 / 64 K-slabs: the reduce runs 2 / 8 / 16 threads
    per output quad combined through LDS.  The [72, 132] output has 2376 quads, which is
    not a multiple of any block's quad count (dead lanes on the last block), on the plain
    and on the transposed (tnarrow) store, with and without accumulate / bias."""
    if kernel == "tnarrow" and with_bias:
        pytest.skip("tnarrow has no bias epilogue")
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(splits)
    R, N, K = 64 * 64, 72, 132                         # reduction rows, output [N, K]
    dy = torch.randn(R, N, device=dev).to(torch.bfloat16)
    a = torch.randn(R, K, device=dev).to(torch.bfloat16)
    dt = torch.float32 if out_f32 else torch.bfloat16
    base = torch.randn(N, K, device=dev).to(dt)
    bias = torch.randn(K, device=dev).to(torch.bfloat16) if with_bias else None
    out = base.clone() if accumulate else torch.empty(N, K, device=dev, dtype=dt)
    NG.gemm(NG.MODE_TN, dy, N, a, K, out, K, N, K, R, bias=bias, accumulate=accumulate, kernel=kernel,
            splits=splits)
    want = dy.float().t() @ a.float()
    if with_bias:
        want = want + bias.float()[None, :]
    if accumulate:
        want = want + base.float()
    assert _rel_err(out, want) < (2e-3 if out_f32 else 1e-2)


@pytest.mark.parametrize("dgrad_nt", [False, True])
def test_linear_dgrad_uses_current_weights_after_flat_optimizer_steps(dgrad_nt, monkeypatch):
    """The NT dgrad's cached W^T must follow the flat optimizer's in-place updates (they
    write the arena behind the parameter views' version counters); the NN dgrad reads W."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_linear
    monkeypatch.setattr(_native_linear, "_DGRAD_NT", dgrad_nt)
    from databricks_distributed_deep_learning_amd.optim import FlatSGD, ParamArena
    torch.manual_seed(4)
    lin = torch.nn.Linear(128, 256).to(dev).to(torch.bfloat16)
    arena = ParamArena(list(lin.named_parameters()))
    opt = FlatSGD(arena, lr=0.5, momentum=0.9)
    for _ in range(3):
        x = torch.randn(1024, 128, device=dev).to(torch.bfloat16).requires_grad_(True)   # M >= 4K: NT dgrad
        y = _native_linear.linear(x, lin.weight, lin.bias, None)
        dy = torch.randn_like(y)
        y.backward(dy)
        want = dy.float() @ lin.weight.detach().float()
        assert _rel_err(x.grad, want) < 2e-2
        opt.step()


def test_conv_dgrad_weight_batch_follows_flat_optimizer_steps():
    """Conv dgrads read their weight layouts from the arena's per-step batch
    (ddl_conv_w_dgrad_batch, one launch per optimizer step): after every flat optimizer step
    (and after an in-place torch update, which bumps only the weight's version) the input
    gradients must use the current weights -- 1x1, stride-1 3x3 and stride-2 (parity classes)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.ops.conv import conv2d_reference
    from databricks_distributed_deep_learning_amd.optim import FlatSGD, ParamArena
    torch.manual_seed(6)
    shapes = {"w1": (64, 1, 1, 32), "w3": (32, 3, 3, 64), "w3s": (48, 3, 3, 32), "w1s": (40, 1, 1, 48)}
    mod = torch.nn.Module()
    for n, s in shapes.items():
        mod.register_parameter(n, torch.nn.Parameter((torch.randn(*s, device=dev) * 0.1).bfloat16()))
    arena = ParamArena(list(mod.named_parameters()))
    opt = FlatSGD(arena, lr=0.5, momentum=0.9)
    plan = [("w1", 1, 0), ("w3", 1, 1), ("w3s", 2, 1), ("w1s", 2, 0)]

    def run(x, ref):
        h = x
        for n, st, pad in plan:
            w = getattr(mod, n)
            h = conv2d_reference(h, w.detach().float(), st, pad) if ref else ops.conv2d(h, w, st, pad)
        return h

    for step in range(4):
        x = torch.randn(4, 16, 16, 32, device=dev).bfloat16().requires_grad_(True)
        y = run(x, False)
        dy = torch.randn_like(y)
        y.backward(dy)
        xr = x.detach().float().requires_grad_(True)
        run(xr, True).backward(dy.float())
        assert _rel_err(x.grad, xr.grad) < 3e-2, step
        if step == 2:
            with torch.no_grad():
                mod.w3.mul_(-1.0)          # torch in-place update: version bump only
        else:
            opt.step()
    cache = getattr(arena, "_ddl_wdg", None)
    assert cache is not None and len(cache.jobs) >= 4 and cache.table is not None


@pytest.mark.parametrize("second_consumer", [False, True])
def test_layernorm_sinks_linear_bias_gradient(second_consumer):
    """LayerNorm backward adds the column sums of its input gradient straight into the
    producing Linear's bias-gradient slot (DataParallel sink); the Linear only marks it ready.
    With a second consumer of the Linear output (autograd sums another gradient into dy) the
    Linear adds the full column sums and takes the LayerNorm's share back out."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    torch.manual_seed(7)
    H = 768
    mod = torch.nn.Module()
    mod.lin = torch.nn.Linear(512, H).to(dev).to(torch.bfloat16)
    mod.ln_w = torch.nn.Parameter(torch.ones(H, device=dev, dtype=torch.bfloat16))
    mod.ln_b = torch.nn.Parameter(torch.zeros(H, device=dev, dtype=torch.bfloat16))
    dp = DataParallel(mod, broadcast_init=False, comm="torch")
    W, b = mod.lin.weight.detach().float(), mod.lin.bias.detach().float()
    scale = torch.linspace(-1, 1, H, device=dev)
    want = torch.zeros(H, device=dev)
    for _ in range(2):                      # second round: accumulation into the slot
        x = torch.randn(2048, 512, device=dev).bfloat16()
        res = torch.randn(2048, H, device=dev).bfloat16()
        y = ops.linear(x, mod.lin.weight, mod.lin.bias, None)
        out = ops.layer_norm(y, mod.ln_w, mod.ln_b, 1e-12, res, 0.0)
        loss = (out.float() * scale).sum()
        if second_consumer:
            loss = loss + (y.float() ** 2).sum() * 1e-3
        loss.backward()
        yr = (x.float() @ W.t() + b).requires_grad_(True)
        lr = (F.layer_norm(yr + res.float(), (H,), eps=1e-12) * scale).sum()
        if second_consumer:
            lr = lr + (yr ** 2).sum() * 1e-3
        lr.backward()
        want += yr.grad.sum(0)
    dp.finish()
    assert getattr(mod.lin.bias, "_ddl_sunk", None) is None
    assert _rel_err(mod.lin.bias.grad, want) < 2e-2


@pytest.mark.parametrize("M,N,K", [(25216, 768, 768), (16384, 2304, 768), (23000, 768, 1536)])
@pytest.mark.parametrize("epi", ["plain", "bias_res", "gelu", "dgelu"])
def test_hybrid_row_split_gemm(M, N, K, epi):
    """256x256-tile GEMMs whose grid ends in a partial round (ViT: 297 tiles on 256 CUs) run
    their last rows split-K (kernel "hybrid", _native_gemm.hybrid_rows): same result as the
    single launch, with the bias / residual / GELU (+ pre-activation) / dGELU epilogues applied
    to both row ranges (the split part's by the reduce kernel)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    hy = NG.hybrid_rows(M, N, K)
    assert hy is not None and 0 < hy[0] < M
    torch.manual_seed(11)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    pre = torch.randn(M, N, device=dev).to(torch.bfloat16)
    for mode in (NG.MODE_NT, NG.MODE_NN):
        wop = w if mode == NG.MODE_NT else w.t().contiguous()     # NN: B[k][n]
        ldb = K if mode == NG.MODE_NT else N
        ref = a.float() @ w.float().t()
        outs = {}
        for kern in ("big", "hybrid"):
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            kw = {}
            if epi == "bias_res":
                kw = dict(bias=b, residual=res)
            elif epi == "gelu":
                kw = dict(bias=b, act="gelu", aux=torch.empty_like(c))
            elif epi == "dgelu":
                kw = dict(act="dgelu", aux=pre)
            NG.gemm(mode, a, K, wop, ldb, c, N, M, N, K, kernel=kern, **kw)
            outs[kern] = (c, kw.get("aux"))
        if epi == "plain":
            exp = ref
        elif epi == "bias_res":
            exp = ref + b.float() + res.float()
        elif epi == "gelu":
            exp = torch.nn.functional.gelu(ref + b.float())
            assert _rel_err(outs["hybrid"][1], ref + b.float()) < 1e-2
        else:
            z = pre.float()
            cdf = 0.5 * (1 + torch.erf(z / 2 ** 0.5))
            exp = ref * (cdf + z * torch.exp(-0.5 * z * z) / (2 * torch.pi) ** 0.5)
        assert _rel_err(outs["hybrid"][0], exp) < 1e-2
        assert _rel_err(outs["hybrid"][0], outs["big"][0].float()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (1000, 576, 200), (4096, 2304, 3072)])
@pytest.mark.parametrize("epi", ["plain", "bias", "bias_res", "relu", "gelu", "dgelu_stats"])
def test_big192_tiles(M, N, K, epi):
    """256 x 192 tiles of the 256x256 kernel (kernel "big192": BERT's N = 768 GEMMs become 256
    tiles instead of 192 on 256 CUs): NT and NN against the fp32 reference for every register
    epilogue, edge tiles (M % 256, K % 64) included, and the dGELU column sums (bias gradient)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(12)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    pre = torch.randn(M, N, device=dev).to(torch.bfloat16)
    for mode in (NG.MODE_NT, NG.MODE_NN):
        wop = w if mode == NG.MODE_NT else w.t().contiguous()
        ldb = K if mode == NG.MODE_NT else N
        ref = a.float() @ w.float().t()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi == "bias":
            kw = dict(bias=b)
        elif epi == "bias_res":
            kw = dict(bias=b, residual=res)
        elif epi == "relu":
            kw = dict(bias=b, act="relu")
        elif epi == "gelu":
            kw = dict(bias=b, act="gelu", aux=torch.empty_like(c))
        elif epi == "dgelu_stats":
            kw = dict(act="dgelu", aux=pre, colstats=torch.zeros(NG.stats_rows_max(M) * 2 * N, device=dev))
        rows = NG.gemm(mode, a, K, wop, ldb, c, N, M, N, K, kernel="big192", **kw)
        exp = ref
        if epi in ("bias", "bias_res", "relu", "gelu"):
            exp = exp + b.float()
        if epi == "bias_res":
            exp = exp + res.float()
        if epi == "relu":
            exp = exp.clamp_min(0)
        if epi == "gelu":
            assert _rel_err(kw["aux"], exp) < 1e-2
            exp = torch.nn.functional.gelu(exp)
        if epi == "dgelu_stats":
            z = pre.float()
            exp = exp * (0.5 * (1 + torch.erf(z / 2 ** 0.5)) + z * torch.exp(-0.5 * z * z) / (2 * torch.pi) ** 0.5)
            sums = kw["colstats"].view(-1, 2, N)[:rows, 0].sum(0)
            assert _rel_err(sums, c.float().sum(0)) < 1e-3
        assert _rel_err(c, exp) < 1e-2, (mode, epi)


@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (1000, 384, 224), (4096, 3072, 768), (2048, 768, 3072)])
@pytest.mark.parametrize("epi", ["plain", "bias", "bias_res", "gelu", "dgelu_stats", "stats"])
def test_duo_kernel(M, N, K, epi):
    """Dual-workgroup 256 x 128 kernel (kernel "duo", gemm_duo.hip): NT and NN against the fp32
    reference for every epilogue it takes, a partial last row tile (M % 256) and odd stage counts
    (K / 32 not a multiple of 3) included; column sums of the stored output (dGELU bias gradient,
    BatchNorm statistics) against the output's own sums."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(13)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    pre = torch.randn(M, N, device=dev).to(torch.bfloat16)
    for mode in (NG.MODE_NT, NG.MODE_NN):
        wop = w if mode == NG.MODE_NT else w.t().contiguous()
        ldb = K if mode == NG.MODE_NT else N
        ref = a.float() @ w.float().t()
        c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi == "bias":
            kw = dict(bias=b)
        elif epi == "bias_res":
            kw = dict(bias=b, residual=res)
        elif epi == "gelu":
            kw = dict(bias=b, act="gelu", aux=torch.empty_like(c))
        elif epi == "dgelu_stats":
            kw = dict(act="dgelu", aux=pre, colstats=torch.zeros(NG.stats_rows_max(M) * 2 * N, device=dev))
        elif epi == "stats":
            kw = dict(colstats=torch.zeros(NG.stats_rows_max(M) * 2 * N, device=dev))
        assert NG._choose(mode, a, K, wop, ldb, c, N, M, N, K, kw.get("bias"), kw.get("act"), kw.get("aux"), None,
                          None, None, False, kw.get("residual"), "duo", kw.get("colstats"))[0] == "duo"
        rows = NG.gemm(mode, a, K, wop, ldb, c, N, M, N, K, kernel="duo", **kw)
        exp = ref
        if epi in ("bias", "bias_res", "gelu"):
            exp = exp + b.float()
        if epi == "bias_res":
            exp = exp + res.float()
        if epi == "gelu":
            assert _rel_err(kw["aux"], exp) < 1e-2
            exp = torch.nn.functional.gelu(exp)
        if epi == "dgelu_stats":
            z = pre.float()
            exp = exp * (0.5 * (1 + torch.erf(z / 2 ** 0.5)) + z * torch.exp(-0.5 * z * z) / (2 * torch.pi) ** 0.5)
        if "stats" in epi:
            st = kw["colstats"].view(-1, 2, N)[:rows]
            assert _rel_err(st[:, 0].sum(0), c.float().sum(0)) < 1e-3
            assert _rel_err(st[:, 1].sum(0), (c.float() ** 2).sum(0)) < 1e-3
        assert not torch.isnan(c.float()).any(), (mode, epi)
        assert _rel_err(c, exp) < 1e-2, (mode, epi)


@pytest.mark.parametrize("N,H,W,C,K,stride", [(2, 28, 28, 128, 128, 1), (2, 56, 56, 128, 128, 2), (3, 14, 14, 256, 256, 1),
                                              (1, 9, 7, 64, 384, 1)])
@pytest.mark.parametrize("epi", ["plain", "stats", "bnb"])
def test_duo_conv(N, H, W, C, K, stride, epi):
    """Implicit-GEMM 3x3 convolution (pad 1) on the dual-workgroup kernel (gemm_duo.hip LCONV): the
    forward against the fp32 reference, its BatchNorm statistics rows, and the BatchNorm-backward
    epilogue (dz = (conv + res) * mask, rows [sum dz | sum dz * xhat])."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    from databricks_distributed_deep_learning_amd.ops._native_conv import _desc
    from databricks_distributed_deep_learning_amd.ops.conv import conv2d_reference
    torch.manual_seed(21)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, 3, 3, C, device=dev) / (3 * C ** 0.5)).to(torch.bfloat16)
    P, Q = (H + 2 - 3) // stride + 1, (W + 2 - 3) // stride + 1
    M = N * P * Q
    desc = _desc(N, H, W, C, P, Q, stride, -1, -1, 1, 1, 3, 3, P, Q)
    ref = conv2d_reference(x.float(), w.float(), stride, 1).reshape(M, K)
    y = torch.full((M, K), float("nan"), device=dev, dtype=torch.bfloat16)
    part = torch.zeros(NG.stats_rows_max(M) * 2 * K, device=dev)
    kw = {}
    if epi == "stats":
        kw = dict(colstats=part)
    elif epi == "bnb":
        xb = (torch.randn(M, K, device=dev) * 2 + 0.5).bfloat16()
        mean = torch.randn(K, device=dev) * 0.3 + 0.5
        istd = torch.rand(K, device=dev) + 0.5
        r = torch.randn(M, K, device=dev).bfloat16()
        mask = torch.randint(0, 256, (M * K // 8,), device=dev, dtype=torch.uint8)
        kw = dict(act="bnb", aux=xb, residual=r, colstats=part, bnb=(mask, mean, istd))
    assert NG._choose(NG.MODE_CONV, x, 0, w, 9 * C, y, K, M, K, 9 * C, None, kw.get("act"), kw.get("aux"), None,
                      desc, None, False, kw.get("residual"), "duo", kw.get("colstats"))[0] == "duo"
    rows = NG.gemm(NG.MODE_CONV, x, 0, w, 9 * C, y, K, M, K, 9 * C, conv=desc, kernel="duo", **kw)
    assert not torch.isnan(y.float()).any()
    if epi == "bnb":
        keep = ((mask[:, None].int() >> torch.arange(8, device=dev)) & 1).view(M, K).bool()
        g = torch.where(keep, ref + r.float(), torch.zeros_like(ref))
        assert _rel_err(y, g) < 1e-2
        dz = y.double()
        sums = part[:rows * 2 * K].view(rows, 2 * K).double().sum(0)
        torch.testing.assert_close(sums[:K], dz.sum(0), rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(sums[K:], (dz * (xb.double() - mean.double()) * istd.double()).sum(0),
                                   rtol=1e-4, atol=1e-3)
        return
    assert _rel_err(y, ref) < 1e-2
    if epi == "stats":
        st = part.view(-1, 2, K)[:rows]
        assert _rel_err(st[:, 0].sum(0), y.float().sum(0)) < 1e-3
        assert _rel_err(st[:, 1].sum(0), (y.float() ** 2).sum(0)) < 1e-3


@pytest.mark.parametrize("M,N,K,splits", [(768, 768, 16384, None), (768, 3072, 4096, 3), (2304, 768, 2048, 1),
                                          (256, 128, 96, 2), (512, 256, 4096, 7), (1024, 128, 8192, 12),
                                          (512, 256, 16384, 40), (256, 256, 32768, 100)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_duo_weight_gradient(M, N, K, splits, accumulate):
    """TN weight gradient on the dual-workgroup kernel (k-outer A staged as two [32 k][128] halves, split-K
    bf16 partial tiles + duo_reduce_k): against the fp32 reference, accumulating into a bf16 gradient."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG
    torch.manual_seed(17)
    dy = torch.randn(K, M, device=dev).to(torch.bfloat16)     # [tokens, out]
    x = torch.randn(K, N, device=dev).to(torch.bfloat16)      # [tokens, in]
    base = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dw = base.clone() if accumulate else torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    ch = NG._choose(NG.MODE_TN, dy, M, x, N, dw, N, M, N, K, None, None, None, splits, None, None, False, None,
                    "duo", None)
    assert ch[0] == "duo"
    NG.gemm(NG.MODE_TN, dy, M, x, N, dw, N, M, N, K, accumulate=accumulate, kernel="duo", splits=splits)
    ref = dy.float().t() @ x.float() + (base.float() if accumulate else 0.)
    assert _rel_err(dw, ref) < 1e-2
