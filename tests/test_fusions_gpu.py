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


@pytest.mark.parametrize("kernel", ["big", "small", "narrow", "duo"])
@pytest.mark.parametrize("M,C,K,res,relu", [(1000, 64, 256, False, True), (4096, 128, 512, True, True),
                                            (777, 256, 64, True, False), (2304, 64, 64, False, True)])
def test_bn_backward_reduction_in_dgrad_epilogue(kernel, M, C, K, res, relu):
    """gemm(act="bnb"): dz = (dy W^T + res) * relu_mask stored, and the per-tile partial rows
    sum to [sum dz | sum dz * xhat] -- the BatchNorm backward's reduction pass."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._native_gemm import MODE_NT, gemm, stats_rows_max
    torch.manual_seed(11)
    dy = torch.randn(M, K, device=dev).bfloat16()
    wt = (torch.randn(C, K, device=dev) * 0.1).bfloat16()
    x = (torch.randn(M, C, device=dev) * 2 + 0.5).bfloat16()
    mean = torch.randn(C, device=dev) * 0.3 + 0.5
    istd = torch.rand(C, device=dev) + 0.5
    r = torch.randn(M, C, device=dev).bfloat16() if res else None
    mask = torch.randint(0, 256, (M * C // 8,), device=dev, dtype=torch.uint8) if relu else None
    rows = stats_rows_max(M)
    part = torch.empty((rows + -(-rows // 32)) * 2 * C, device=dev)
    out = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    nrows = gemm(MODE_NT, dy, K, wt, K, out, C, M, C, K, act="bnb", aux=x, residual=r, colstats=part,
                 bnb=(mask, mean, istd), kernel=kernel)
    g = dy.float() @ wt.float().t() + (r.float() if res else 0.)
    if relu:
        keep = ((mask[:, None].int() >> torch.arange(8, device=dev)) & 1).view(M, C).bool()
        g = torch.where(keep, g, torch.zeros_like(g))
    assert ((out.float() - g).abs().max() / g.abs().max()).item() < 1e-2
    dz = out.float()
    sums = part[:nrows * 2 * C].view(nrows, 2 * C).double().sum(0)
    ref_s = dz.double().sum(0)
    ref_q = (dz.double() * (x.double() - mean.double()) * istd.double()).sum(0)
    torch.testing.assert_close(sums[:C], ref_s, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(sums[C:], ref_q, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_bn_backward_epilogue_model_gradients(arch):
    """ResNet gradients with the BN backward reduction fused into the dgrad epilogues equal
    those of the separate partial pass (same dz values, different summation order)."""
    import copy
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import models, ops
    from databricks_distributed_deep_learning_amd.models.layers import cast_params
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC, _native_norm as NN
    torch.manual_seed(0)
    m = cast_params(getattr(models, arch)(num_classes=10), torch.bfloat16).to(dev).train()
    x = torch.randn(8, 64, 64, 3, device=dev, dtype=torch.bfloat16)
    y = torch.randint(0, 10, (8,), device=dev)
    grads = {}
    saved = (NC._BN_BWD_EPI, NC._BN_BWD_EPI_RES, NN._BN_BWD_EPI)
    for flag in (True, False):
        # fused run: every eligible dgrad, the residual-adding ones included
        NC._BN_BWD_EPI = NC._BN_BWD_EPI_RES = NN._BN_BWD_EPI = flag
        try:
            mm = copy.deepcopy(m)
            ops.cross_entropy(mm(x).float(), y).backward()
            grads[flag] = {n: q.grad.float() for n, q in mm.named_parameters() if q.grad is not None}
        finally:
            NC._BN_BWD_EPI, NC._BN_BWD_EPI_RES, NN._BN_BWD_EPI = saved
    assert grads[True].keys() == grads[False].keys() and len(grads[True]) > 20
    rel = {n: ((grads[True][n] - grads[False][n]).norm() / grads[False][n].norm().clamp_min(1e-12)).item()
           for n in grads[True]}
    # one summation-order difference per BN, amplified through the (random-init) depth:
    # tight near the loss, loose at the stem
    for n, e in rel.items():
        assert e < (3e-2 if n.startswith(("layer3.", "layer4.", "fc.")) else 0.15), (n, e)


@pytest.mark.parametrize("shape", [(8, 28, 28, 256), (4, 14, 14, 512), (6, 7, 7, 2048)])
def test_downsample_block_dual_bn_apply(shape):
    """relu(BN(y) + BN2(y2)) in one pass (ddl_bn_apply2, a downsample block's output): output,
    input / affine gradients and running statistics equal the two separate BatchNorms."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(5)
    C = shape[-1]
    y = torch.randn(*shape, device=dev).bfloat16()
    y2 = (torch.randn(*shape, device=dev) * 2 + 0.5).bfloat16()
    dout = torch.randn(*shape, device=dev).bfloat16()
    prm = [(torch.rand(C, device=dev) + 0.5).bfloat16(), (torch.randn(C, device=dev) * 0.1).bfloat16(),
           (torch.rand(C, device=dev) + 0.5).bfloat16(), (torch.randn(C, device=dev) * 0.1).bfloat16()]
    res = []
    for fused in (True, False):
        a, a2 = y.clone().requires_grad_(True), y2.clone().requires_grad_(True)
        g, b, g2, b2 = (t.clone().requires_grad_(True) for t in prm)
        rm, rv, rm2, rv2 = (torch.zeros(C, device=dev), torch.ones(C, device=dev),
                            torch.zeros(C, device=dev), torch.ones(C, device=dev))
        if fused:
            out = ops.batch_norm_add_bn(a, g, b, rm, rv, 0.1, 1e-5, a2, g2, b2, rm2, rv2, 0.1, 1e-5)
            assert out is not None
        else:
            r = ops.batch_norm(a2, g2, b2, rm2, rv2, True, 0.1, 1e-5, False, None)
            out = ops.batch_norm(a, g, b, rm, rv, True, 0.1, 1e-5, True, r)
        out.backward(dout)
        res.append([out.float(), a.grad.float(), a2.grad.float(), g.grad.float(), b.grad.float(), g2.grad.float(),
                    b2.grad.float(), rm, rv, rm2, rv2])
    names = ["out", "dy", "dy2", "dg", "db", "dg2", "db2", "rm", "rv", "rm2", "rv2"]
    for n, u, v in zip(names, res[0], res[1]):
        if n in ("out", "rm", "rv", "rm2", "rv2"):
            torch.testing.assert_close(u, v, rtol=2e-2, atol=2e-2, msg=n)
        else:
            # the fused pass adds BN2's output unrounded, so ReLU-mask bits at |t| < ~1 bf16 ulp
            # differ from the bf16-residual path (~2 % of the gradient norm at these sizes; a
            # dropped or misrouted term would be O(1)): compare gradients by relative norm
            assert ((u - v).norm() / v.norm().clamp_min(1e-12)).item() < 5e-2, n


@pytest.mark.parametrize("fused_bwd", [False, True])
@pytest.mark.parametrize("shape", [(4, 112, 112, 64), (3, 30, 18, 16)])
def test_stem_bn_relu_maxpool(shape, fused_bwd, monkeypatch):
    """maxpool3x3/2(relu(BN(x))) in one pass (ddl_bn_relu_maxpool): pooled output equal to BN
    apply -> max-pool (the same bf16-rounded activations are pooled), gradients and running
    statistics equal."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.ops import _native_norm
    monkeypatch.setattr(_native_norm, "_FUSED_STEM_BWD", fused_bwd)   # max-pool gather inside the BN backward
    torch.manual_seed(6)
    C = shape[-1]
    x = torch.randn(*shape, device=dev).bfloat16()
    g0, b0 = (torch.rand(C, device=dev) + 0.5).bfloat16(), (torch.randn(C, device=dev) * 0.3).bfloat16()
    res = []
    for fused in (True, False):
        a = x.clone().requires_grad_(True)
        g, b = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        if fused:
            out = ops.bn_relu_maxpool(a, g, b, rm, rv, 0.1, 1e-5)
            assert out is not None
        else:
            out = ops.max_pool2d(ops.batch_norm(a, g, b, rm, rv, True, 0.1, 1e-5, True, None), 3, 2, 1)
        torch.manual_seed(0)
        out.backward(torch.randn(out.shape, device=dev).bfloat16())
        res.append((out.float(), a.grad.float(), g.grad.float(), b.grad.float(), rm, rv))
    assert torch.equal(res[0][0], res[1][0])
    for n, u, v in zip(["dx", "dg", "db"], res[0][1:4], res[1][1:4]):
        assert ((u - v).norm() / v.norm().clamp_min(1e-12)).item() < 1e-2, n
    torch.testing.assert_close(res[0][4], res[1][4])
    torch.testing.assert_close(res[0][5], res[1][5])


@pytest.mark.parametrize("nblk,C", [(300, 64), (3000, 512), (1057, 2048), (128, 256), (129, 64), (20000, 64), (1, 64),
                                    (2, 256), (5, 2048), (64, 128)])
def test_bn_finalize_from_many_partial_rows(nblk, C):
    """Many GEMM-epilogue partial rows -> BatchNorm forward statistics and backward coefficients
    (the merged multi-workgroup finalize: 128-row slices + last-arriver combine; 129 rows = a
    one-row last slice, 20000 = more rows than 128 slices of 128), against fp64 sums of the same
    rows, and bit-identical over repeated launches (fixed summation order, tickets re-armed)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._lib import call, p
    torch.manual_seed(5)
    M = nblk * 128
    part = torch.rand(nblk, 2 * C, device=dev) * 4.0
    part[:, C:] += part[:, :C] ** 2 / 16        # second moments >= mean^2 on average
    ws = torch.empty(-(-nblk // 32) * 2 * C, device=dev)
    gamma = (torch.rand(C, device=dev) + 0.5).bfloat16()
    beta = torch.randn(C, device=dev).bfloat16()
    s, q = part.double().sum(0)[:C], part.double().sum(0)[C:]
    first = None
    for rep in range(3):
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        st = torch.empty(4, C, device=dev)
        call("ddl_bn_fwd_from_partials", 1, p(part), nblk, M, C, p(gamma), p(beta), p(rm), p(rv), 0.1, 1e-5,
             p(st[0]), p(st[1]), p(st[2]), p(st[3]), p(ws), ws.numel())
        mean = s / M
        var = (q / M - mean * mean).clamp_min(0)
        torch.testing.assert_close(st[0].double(), mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(st[1].double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(rm.double(), 0.1 * mean, rtol=1e-5, atol=1e-6)
        if first is None:
            first = st.clone()
        assert torch.equal(st, first), "finalize not deterministic across launches"
    # backward: coefficients (k1, mean dz, mean dz*xhat) and dgamma / dbeta from the same rows
    x = torch.randn(M, C, device=dev).bfloat16()
    dz = torch.randn(M, C, device=dev).bfloat16()
    istd = torch.rand(C, device=dev) + 0.5
    mu = torch.randn(C, device=dev) * 0.1
    coef = torch.empty(3 * C, device=dev)
    dg, db = torch.empty(C, device=dev).bfloat16(), torch.empty(C, device=dev).bfloat16()
    dx = torch.empty_like(x)
    call("ddl_bn_bwd_from_partials", 1, p(part), nblk, p(ws), ws.numel(), p(dz), p(x), p(mu), p(istd), p(gamma), M, C,
         p(dg), p(db), p(coef), p(dx), None, 0)
    torch.testing.assert_close(coef[C:2 * C].double(), s / M, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(coef[2 * C:].double(), q / M, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(db.double(), s.to(torch.bfloat16).double(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dg.double(), q.to(torch.bfloat16).double(), rtol=1e-2, atol=1e-2)
    k1 = gamma.float() * istd
    ref = k1 * (dz.float() - coef[C:2 * C] - (x.float() - mu) * istd * coef[2 * C:])
    assert ((dx.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("C", [4160, 8192])
def test_bn_finalize_wider_than_ticket_window(C):
    """a merged finalize launch owns 64 arrival tickets (one per 64 channels).  Layers
    wider than 4096 channels must take the collapse path instead of indexing past their window
    (into the next launch's tickets, or past the pool on the last window).  Checked against fp64,
    then a narrow merged finalize on every remaining window must still be exact and repeatable
    (a stray ticket would leave a window's counter non-zero and skip a channel group's finish)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._lib import call, p
    torch.manual_seed(7)
    nblk = 600
    M = nblk * 128
    part = torch.rand(nblk, 2 * C, device=dev) * 4.0
    ws = torch.empty(-(-nblk // 32) * 2 * C, device=dev)
    gamma = torch.ones(C, device=dev).bfloat16()
    beta = torch.zeros(C, device=dev).bfloat16()
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    st = torch.empty(4, C, device=dev)
    call("ddl_bn_fwd_from_partials", 1, p(part), nblk, M, C, p(gamma), p(beta), p(rm), p(rv), 0.1, 1e-5,
         p(st[0]), p(st[1]), p(st[2]), p(st[3]), p(ws), ws.numel())
    torch.testing.assert_close(st[0].double(), part.double().sum(0)[:C] / M, rtol=1e-5, atol=1e-6)
    c2, n2 = 4096, 300
    part2 = torch.rand(n2, 2 * c2, device=dev)
    ws2 = torch.empty(-(-n2 // 32) * 2 * c2, device=dev)
    g2, b2 = torch.ones(c2, device=dev).bfloat16(), torch.zeros(c2, device=dev).bfloat16()
    want = part2.double().sum(0)[:c2] / (n2 * 128)
    first = None
    for _ in range(8192 // 64 + 2):            # every window of the ticket pool, and around again
        st2 = torch.empty(4, c2, device=dev)
        call("ddl_bn_fwd_from_partials", 1, p(part2), n2, n2 * 128, c2, p(g2), p(b2), p(torch.zeros(c2, device=dev)),
             p(torch.ones(c2, device=dev)), 0.1, 1e-5, p(st2[0]), p(st2[1]), p(st2[2]), p(st2[3]), p(ws2), ws2.numel())
        first = st2.clone() if first is None else first
        assert torch.equal(st2, first)
    torch.testing.assert_close(first[0].double(), want, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("nrows,width,n,acc", [(100, 1536, 768, 1), (777, 64, 64, 0), (2000, 6144, 3072, 1)])
def test_rows_sum_sink_many_rows(nrows, width, n, acc):
    """Column sums of many partial rows straight into a bf16 gradient slot (a Linear's bias),
    against fp64."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._lib import call, p
    torch.manual_seed(2)
    part = torch.randn(nrows, width, device=dev)
    ws = torch.empty(-(-nrows // 32) * width, device=dev)
    sink = torch.randn(n, device=dev).bfloat16()
    before = sink.double().clone()
    for _ in range(2):
        out = sink.clone()
        call("ddl_rows_sum_sink", 1, p(part), nrows, width, n, p(out), acc, p(ws))
        ref = part.double().sum(0)[:n] + (before if acc else 0)
        torch.testing.assert_close(out.double(), ref.to(torch.bfloat16).double(), rtol=2e-2, atol=2e-2)
