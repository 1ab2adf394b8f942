"""Numerics of the HIP kernels against plain-PyTorch fp32 references (GPU only)."""
import pytest
import torch
import torch.nn.functional as F

from conftest import gpu_device

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{what}: max err {err:.3e} > tol {tol:.3e}"


def _native_lib_loaded():
    from databricks_distributed_deep_learning_amd.ops import _lib
    assert _lib.available(), _lib.load_error()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("C", [64, 256, 2048, 24])
@pytest.mark.parametrize("big", [False, True])
def test_batchnorm_train(dtype, relu, res, C, big):
    if big and (dtype == torch.float32 or C == 24):
        pytest.skip("large-M case: bf16 row-major paths only")
    dev = gpu_device()
    _native_lib_loaded()
    from databricks_distributed_deep_learning_amd.ops import norm
    torch.manual_seed(0)
    # big: enough rows that every thread of the row-major BN kernels runs its
    # 4-rows-in-flight loop (M > 4 * 2048 blocks * rows per block)
    N, H, W = ((16, 130, 130) if C <= 256 else (4, 60, 60)) if big else (4, 7, 9)
    x = (torch.randn(N, H, W, C, device=dev) * 2 + 0.5).to(dtype)
    r = torch.randn(N, H, W, C, device=dev).to(dtype) if res else None
    g = (torch.rand(C, device=dev) + 0.5).to(dtype)
    b = (torch.randn(C, device=dev) * 0.1).to(dtype)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm.clone(), rv.clone()
    xs = [x.clone().requires_grad_(True), x.float().clone().requires_grad_(True)]
    gs = [g.clone().requires_grad_(True), g.float().clone().requires_grad_(True)]
    bs = [b.clone().requires_grad_(True), b.float().clone().requires_grad_(True)]
    rs = [r.clone().requires_grad_(True), r.float().clone().requires_grad_(True)] if res else [None, None]
    y = norm.batch_norm(xs[0], gs[0], bs[0], rm, rv, True, 0.1, 1e-5, relu, rs[0])
    # Reference without the ReLU; the ReLU is applied with the NATIVE output's mask
    # so elements whose pre-activation rounds to the other side of 0 cannot flip.
    yr = norm.batch_norm_reference(xs[1], gs[1], bs[1], rm2, rv2, True, 0.1, 1e-5, False, rs[1])
    if relu:
        yr = yr * (y.detach() > 0).float()
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    keep = (y.detach() > 0) | (yr.detach().abs() > 0) if relu else torch.ones_like(yr, dtype=torch.bool)
    _close(y.float()[keep], yr[keep], tol, tol, "bn fwd")
    _close(rm, rm2, 1e-4, 1e-3, "running_mean")
    _close(rv, rv2, 1e-4, 1e-3, "running_var")
    dy = torch.randn_like(yr)
    y.backward(dy.to(dtype))
    yr.backward(dy)
    _close(xs[0].grad, xs[1].grad, tol, tol, "bn dx")
    _close(gs[0].grad, gs[1].grad, tol * 10, tol * 10, "bn dgamma")
    _close(bs[0].grad, bs[1].grad, tol * 10, tol * 10, "bn dbeta")
    if res:
        _close(rs[0].grad, rs[1].grad, tol, tol, "bn dres")


def _hash_keep(seed: int, n: int, p: float):
    """Python replica of the kernels' dropout RNG (ddl_common.h pair_hash / keep_half):
    one lowbias32 round per pair of element indices, 16 bits per element."""
    import numpy as np

    def lowbias32(x):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7feb352d)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846ca68b)
        return x ^ (x >> np.uint32(16))
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64)
        pidx = idx >> np.uint64(1)
        lo = (pidx & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (pidx >> np.uint64(32)).astype(np.uint32)
        x = (lo ^ np.uint32(seed & 0xFFFFFFFF)) + hi * np.uint32(0x9E3779B9) + np.uint32(seed >> 32)
        h = lowbias32(x)
        half = (h >> ((idx & np.uint64(1)).astype(np.uint32) * np.uint32(16))) & np.uint32(0xFFFF)
    thresh = min(65536, int(p * 65536.0))
    return torch.from_numpy(half.astype(np.int64) >= thresh)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H", [768, 1024])
def test_layernorm_fused_dropout(dtype, H):
    """LN(dropout(Linear(x)) + res) with the dropout fused into the LN kernels, against
    an fp32 reference that rebuilds the mask from the same counter hash: forward, x /
    residual / gamma / beta gradients and the producing Linear's bias gradient (taken
    from the LN backward's column sums of the masked gradient)."""
    dev = gpu_device()
    _native_lib_loaded()
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.ops import norm
    torch.manual_seed(2)
    B, S, pdrop = 4, 64, 0.1
    x = torch.randn(B, S, H, device=dev).to(dtype)
    w = (torch.randn(H, H, device=dev) / H ** 0.5).to(dtype)
    lb = (torch.randn(H, device=dev) * 0.1).to(dtype)
    g = (torch.rand(H, device=dev) + 0.5).to(dtype)
    b = (torch.randn(H, device=dev) * 0.1).to(dtype)
    r = torch.randn(B, S, H, device=dev).to(dtype)
    leaves = lambda ts: [t.clone().requires_grad_(True) for t in ts]  # noqa: E731
    a = leaves([x, w, lb, g, b, r])
    f = leaves([t.float() for t in (x, w, lb, g, b, r)])
    torch.manual_seed(123)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())     # what the op will draw (new_seed)
    torch.manual_seed(123)
    y = norm.layer_norm(ops.linear(a[0], a[1], a[2], None), a[3], a[4], 1e-12, a[5], dropout=pdrop)
    keep = _hash_keep(seed, B * S * H, pdrop).to(dev).view(B, S, H)
    assert 0.85 < keep.float().mean().item() < 0.95
    hidden = (f[0] @ f[1].t() + f[2]) * keep / (1 - pdrop)
    yr = norm.layer_norm_reference(hidden, f[3], f[4], 1e-12, f[5])
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    _close(y, yr, tol, tol, "ln+dropout fwd")
    dy = torch.randn_like(yr)
    y.backward(dy.to(dtype))
    yr.backward(dy)
    _close(a[0].grad, f[0].grad, tol, tol, "dx")
    _close(a[2].grad, f[2].grad, tol * 20, tol, "linear bias grad (LN column sums)")
    _close(a[3].grad, f[3].grad, tol * 20, tol, "dgamma")
    _close(a[4].grad, f[4].grad, tol * 20, tol, "dbeta")
    _close(a[5].grad, f[5].grad, tol * 10, tol, "dres")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H", [768, 1024])
@pytest.mark.parametrize("res", [None, "full", "bcast"])
@pytest.mark.parametrize("B,S", [(3, 37), (64, 197)])   # 64 x 197 rows: > 64 partial rows (merged finish)
def test_layernorm(dtype, H, res, B, S):
    dev = gpu_device()
    _native_lib_loaded()
    from databricks_distributed_deep_learning_amd.ops import norm
    torch.manual_seed(1)
    x = torch.randn(B, S, H, device=dev).to(dtype)
    g = (torch.rand(H, device=dev) + 0.5).to(dtype)
    b = (torch.randn(H, device=dev) * 0.1).to(dtype)
    r = None
    if res == "full":
        r = torch.randn(B, S, H, device=dev).to(dtype)
    elif res == "bcast":
        r = torch.randn(1, S, H, device=dev).to(dtype)
    leaves = lambda t: None if t is None else t.clone().requires_grad_(True)  # noqa: E731
    a = [leaves(x), leaves(g), leaves(b), leaves(r)]
    f = [leaves(x.float()), leaves(g.float()), leaves(b.float()), leaves(None if r is None else r.float())]
    y = norm.layer_norm(a[0], a[1], a[2], 1e-12, a[3])
    yr = norm.layer_norm_reference(f[0], f[1], f[2], 1e-12, f[3])
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    _close(y, yr, tol, tol, "ln fwd")
    dy = torch.randn_like(yr)
    y.backward(dy.to(dtype))
    yr.backward(dy)
    _close(a[0].grad, f[0].grad, tol, tol, "ln dx")
    _close(a[1].grad, f[1].grad, tol * 20, tol, "ln dgamma")
    _close(a[2].grad, f[2].grad, tol * 20, tol, "ln dbeta")
    if r is not None:
        _close(a[3].grad, f[3].grad, tol * 10, tol, "ln dres")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gelu_dropout(dtype):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_elementwise as E
    x = torch.randn(4096, 96, device=dev).to(dtype).requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    y = E.gelu(x)
    yr = F.gelu(xr)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    _close(y, yr, tol, tol, "gelu")
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    _close(x.grad, xr.grad, tol * 2, tol, "gelu bwd")
    # dropout: keep-rate and scaling; backward reuses the same mask
    ones = torch.ones(1 << 20, device=dev, dtype=dtype, requires_grad=True)
    d = E.dropout(ones, 0.1)
    kept = (d != 0).float().mean().item()
    assert abs(kept - 0.9) < 0.005
    _close(d[d != 0], torch.full_like(d[d != 0], 1 / 0.9), 1e-2)
    d.backward(torch.ones_like(d))
    assert torch.equal(ones.grad != 0, d != 0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [2, 1000])
def test_cross_entropy(dtype, C):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_loss as L
    logits = (torch.randn(64, C, device=dev) * 3).to(dtype).requires_grad_(True)
    lr = logits.detach().float().requires_grad_(True)
    y = torch.randint(0, C, (64,), device=dev)
    loss = L.cross_entropy(logits, y)
    ref = F.cross_entropy(lr, y)
    _close(loss, ref, 1e-3 if dtype == torch.bfloat16 else 1e-5, 1e-3)
    (loss * 2).backward()
    (ref * 2).backward()
    _close(logits.grad, lr.grad, 1e-3, 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_pools(dtype):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_pool as Pn, pool
    x = torch.randn(2, 15, 13, 64, device=dev).to(dtype).requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    y = Pn.max_pool2d(x, 3, 2, 1)
    yr = pool.max_pool2d_reference(xr, 3, 2, 1)
    _close(y, yr, 0.0, 0.0, "maxpool fwd")
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g.to(dtype).float())
    _close(x.grad, xr.grad, 1e-6, 1e-2 if dtype == torch.bfloat16 else 1e-6, "maxpool bwd")
    z = torch.randn(4, 7, 7, 256, device=dev).to(dtype).requires_grad_(True)
    zr = z.detach().float().requires_grad_(True)
    a = Pn.global_avg_pool(z)
    ar = zr.mean(dim=(1, 2))
    _close(a, ar, 1e-2 if dtype == torch.bfloat16 else 1e-6)
    g = torch.randn_like(ar)
    a.backward(g.to(dtype))
    ar.backward(g)
    _close(z.grad, zr.grad, 1e-3)


def test_embedding():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_embedding as Em
    w = torch.randn(1000, 768, device=dev, dtype=torch.bfloat16, requires_grad=True)
    wr = w.detach().float().requires_grad_(True)
    ids = torch.randint(0, 1000, (8, 128), device=dev)
    y = Em.embedding(ids, w)
    yr = F.embedding(ids, wr)
    _close(y, yr, 0.0)
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    _close(w.grad, wr.grad, 5e-2, 1e-2)


@pytest.mark.parametrize("V,D,n,skew", [
    (1000, 768, 1024, "uniform"),     # short runs, chunk edges everywhere
    (30522, 768, 16384, "padding"),   # one id (padding) over ~half the positions: a run across hundreds of chunks
    (2, 768, 4096, "uniform"),        # token types: two runs of ~2048
    (50, 1024, 1001, "runs16"),       # runs of exactly one chunk, n not a multiple of 16
    (7, 64, 37, "uniform"),           # D = 64: one half-used column slab
])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_backward_sorted_deterministic(V, D, n, skew, dtype):
    """Sorted segmented-sum embedding backward (ddl_embedding_bwd_sorted): every id's rows summed in
    token order against fp32 index_add_, including runs that cross many 16-position chunks; the
    accumulate form adds to a gradient slot and leaves untouched rows alone; two runs are bitwise equal."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._lib import call, dcode, p
    torch.manual_seed(1)
    ids = torch.randint(0, V, (n,), device=dev)
    if skew == "padding":
        ids[torch.rand(n, device=dev) < 0.5] = 0
    elif skew == "runs16":
        ids = (torch.arange(n, device=dev) // 16) % V
        ids = ids[torch.randperm(n, device=dev)]
    dy = torch.randn(n, D, device=dev).to(dtype)
    ref = torch.zeros(V, D, device=dev, dtype=torch.float64).index_add_(0, ids, dy.double())
    s, pi = torch.sort(ids.to(torch.int32), stable=True)
    part = torch.empty(2 * ((n + 15) // 16) * D, dtype=torch.float32, device=dev)
    outs = []
    for acc in (0, 0, 1):
        base = torch.randn(V, D, device=dev).to(dtype) if acc else torch.zeros(V, D, device=dev, dtype=dtype)
        dw = base.clone()
        call("ddl_embedding_bwd_sorted", dcode(dy), p(s), p(pi), p(dy), p(dw), p(part), n, D, acc)
        torch.cuda.synchronize()
        outs.append((base, dw))
    assert torch.equal(outs[0][1], outs[1][1])
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    got = outs[0][1].double()
    assert ((got - ref).abs().max() / ref.abs().max()).item() < tol
    base, dw = outs[2]
    touched = torch.zeros(V, dtype=torch.bool, device=dev)
    touched[ids] = True
    assert torch.equal(dw[~touched], base[~touched])
    want = base.double() + ref
    assert ((dw.double() - want).abs().max() / want.abs().max()).item() < tol


def test_embedding_backward_sorted_matches_atomic_path(monkeypatch):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_embedding as Em
    torch.manual_seed(2)
    w = torch.randn(3000, 768, device=dev, dtype=torch.bfloat16)
    ids = torch.randint(0, 3000, (16, 128), device=dev)
    ids[:, 100:] = 0
    g = torch.randn(16, 128, 768, device=dev, dtype=torch.bfloat16)
    grads = {}
    for flag in (True, False):
        monkeypatch.setattr(Em, "_SORTED", flag)
        ww = w.clone().requires_grad_(True)
        Em.embedding(ids, ww).backward(g)
        grads[flag] = ww.grad.float()
    assert ((grads[True] - grads[False]).abs().max() / grads[False].abs().max()).item() < 1e-2


@pytest.mark.parametrize("name", ["sgd", "adamw", "lamb"])
@pytest.mark.parametrize("pdtype", [torch.float32, torch.bfloat16])
def test_flat_optimizers_match_torch_path(name, pdtype):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.config import TrainConfig
    from databricks_distributed_deep_learning_amd.ops import _lib
    from databricks_distributed_deep_learning_amd.optim import ParamArena, build_optimizer

    def make():
        torch.manual_seed(3)
        m = torch.nn.Sequential(torch.nn.Linear(67, 129), torch.nn.LayerNorm(129), torch.nn.Linear(129, 5)).to(dev)
        for prm in m.parameters():
            prm.data = prm.data.to(pdtype)
        return m

    cfg = TrainConfig(lr=1e-2, weight_decay=0.1, momentum=0.9, max_grad_norm=1.0 if name == "lamb" else 0.0)
    outs = []
    for mode in ("auto", "off"):
        _lib.set_mode(mode)
        m = make()
        arena = ParamArena(list(m.named_parameters()))
        opt = build_optimizer(name, arena, cfg)
        g = torch.Generator(device=dev).manual_seed(7)
        pad_mask = torch.zeros(arena.numel, dtype=torch.bool, device=dev)
        for e in arena.entries:
            pad_mask[e.offset:e.offset + e.numel] = True
        for _ in range(3):
            # real gradients are zero in the alignment padding between tensors
            arena.grad.copy_((torch.randn(arena.numel, generator=g, device=dev) * pad_mask).to(pdtype))
            opt.step(arena.grad, grad_scale=0.5)
        outs.append((opt.params32.clone(), arena.flat.clone()))
    _lib.set_mode("auto")
    _close(outs[0][0], outs[1][0], 1e-5, 1e-5, f"{name} master")
    _close(outs[0][1], outs[1][1], 1e-2 if pdtype == torch.bfloat16 else 1e-5, 1e-5, f"{name} param")


@pytest.mark.parametrize("name", ["sgd", "adamw", "lamb"])
def test_sharded_flat_optimizers_match_torch_path(name, monkeypatch):
    """ZeRO-1 rank 0 of 2 owning chunk 0 of two buckets (local index space, per-row arena
    offsets in the block table): native kernels == torch path on the owned elements; the
    unowned arena elements are left alone (the all-gather is stubbed out)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.config import TrainConfig
    from databricks_distributed_deep_learning_amd.ops import _lib
    from databricks_distributed_deep_learning_amd.optim import ParamArena, build_optimizer
    from databricks_distributed_deep_learning_amd.optim import flat as F_
    monkeypatch.setattr(F_, "_sum_over_ranks", lambda t: None)

    def make():
        torch.manual_seed(3)
        m = torch.nn.Sequential(torch.nn.Linear(67, 129), torch.nn.LayerNorm(129), torch.nn.Linear(129, 5)).to(dev)
        for prm in m.parameters():
            prm.data = prm.data.to(torch.bfloat16)
        return m

    cfg = TrainConfig(lr=1e-2, weight_decay=0.1, momentum=0.9, max_grad_norm=1.0 if name == "lamb" else 0.0)
    outs = []
    for mode in ("auto", "off"):
        _lib.set_mode(mode)
        m = make()
        arena = ParamArena(list(m.named_parameters()), pad_multiple=128)
        split = (arena.numel // 2) // 128 * 128
        opt = build_optimizer(name, arena, cfg, shard=(0, 2, [(0, split), (split, arena.numel)]))
        opt.gather_fn = lambda groups, ranges: None
        before = arena.flat.clone()
        pad_mask = torch.zeros(arena.numel, dtype=torch.bool, device=dev)
        for e in arena.entries:
            pad_mask[e.offset:e.offset + e.numel] = True
        lmask = opt._local(pad_mask)        # gradients are zero in the alignment padding
        g = torch.Generator(device=dev).manual_seed(7)
        for _ in range(3):
            local = (torch.randn(opt.state_numel, generator=g, device=dev) * lmask).to(torch.bfloat16)
            opt.step(local, grad_scale=0.5)
        owned = torch.zeros(arena.numel, dtype=torch.bool, device=dev)
        for lo, hi, _ in opt.ranges:
            owned[lo:hi] = True
        assert torch.equal(arena.flat[~owned], before[~owned])
        outs.append((opt.params32.clone(), arena.flat[owned].clone()))
    _lib.set_mode("auto")
    _close(outs[0][0], outs[1][0], 1e-5, 1e-5, f"{name} sharded master")
    _close(outs[0][1], outs[1][1], 1e-2, 1e-5, f"{name} sharded param")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,k", [(1, 1000, 5), (3, 1000, 5), (4, 37, 3), (2, 4096, 10)])
def test_softmax_topk(dtype, B, C, k):
    """Inference post-processing kernel (softmax + top-k, the reference's top-5)."""
    dev = gpu_device()
    _native_lib_loaded()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(5)
    logits = (torch.randn(B, C, device=dev) * 3).to(dtype)
    p, v, i = ops.softmax_topk(logits, k)
    pr = torch.softmax(logits.float(), -1)
    vr, ir = torch.topk(pr, k, -1)
    _close(p, pr, 1e-6, 1e-5, "probs")
    _close(v, vr, 1e-6, 1e-5, "top-k values")
    # indices: equal wherever the reference values are distinct
    assert torch.equal(i, ir) or torch.allclose(pr.gather(-1, i), vr, atol=1e-7)


@pytest.mark.parametrize("K,R,S,C,rs,ss", [(64, 3, 3, 64, [2, 1, 0], [2, 1, 0]), (256, 1, 1, 1024, [0], [0]),
                                           (48, 3, 3, 40, [1], [0, 2]), (2048, 1, 1, 512, [0], [0]),
                                           (70, 7, 7, 33, [6, 4, 2, 0], [5, 3, 1])])
def test_conv_dgrad_weight_layout(K, R, S, C, rs, ss):
    """ddl_conv_w_dgrad: out[c][r'][s'][k] = w[k][rs[r']][ss[s']][c] (tiled transpose, odd tails)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._native_conv import _w_dgrad
    w = torch.randn(K, R, S, C, device=dev).bfloat16()
    out = _w_dgrad(w, rs, ss)
    ref = w[:, rs][:, :, ss].permute(3, 1, 2, 0).contiguous()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("B,H,P,D", [(4, 224, 16, 768), (3, 64, 16, 256), (2, 32, 8, 64)])
def test_patch_embed_implicit_im2col(B, H, P, D):
    """ViT patch embedding as an implicit-im2col GEMM on the NHWC image (no patchify copy)
    == patchify + Linear in fp32, forward and weight / bias gradients (arena sinks)."""
    dev = gpu_device()
    _native_lib_loaded()
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    torch.manual_seed(2)
    x = torch.randn(B, H, H, 3, device=dev).bfloat16()
    w = (torch.randn(D, P * P * 3, device=dev) * 0.05).bfloat16().requires_grad_(True)
    b = (torch.randn(D, device=dev) * 0.1).bfloat16().requires_grad_(True)
    y = NC.patch_embed(x, w, b, P)
    assert y is not None
    xr = x.float().view(B, H // P, P, H // P, P, 3).permute(0, 1, 3, 2, 4, 5).reshape(B, (H // P) ** 2, P * P * 3)
    wr, br = w.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    yr = xr @ wr.t() + br
    _close(y, yr, 2e-2, 1e-2, "patch embed fwd")
    g = torch.randn_like(yr).bfloat16()
    y.backward(g)
    yr.backward(g.float())
    _close(w.grad, wr.grad, 3e-2, 1e-2, "patch embed dW")
    _close(b.grad, br.grad, 3e-2, 1e-2, "patch embed db")
    assert ops.patch_embed(x, w, b, P).shape == (B, (H // P) ** 2, D)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_acc_grad(dtype):
    """Grad-accumulation pass (ddl_acc_grad): acc32 = g (first micro-step: no zero fill, the old
    contents unread) or acc32 += g, g = 0 on a micro-step's drain and left as is on the last pass --
    against the fp32 reference."""
    dev = gpu_device()
    _native_lib_loaded()
    from databricks_distributed_deep_learning_amd.parallel.ddp import _acc_grad
    torch.manual_seed(0)
    n = 3 * 8192 + 40
    for first in (True, False):
        for zero in (True, False):
            g = torch.randn(n, device=dev).to(dtype)
            acc = torch.full((n,), float("nan"), device=dev) if first else torch.randn(n, device=dev)
            ref = g.float().clone() if first else acc + g.float()
            g0 = g.clone()
            _acc_grad(acc, g, first=first, zero_grad=zero)
            torch.cuda.synchronize()
            assert torch.equal(acc, ref)
            assert (not g.any()) if zero else torch.equal(g, g0)


def test_no_sync_fp32_accumulation_over_steps():
    """DataParallel.no_sync with accumulate_fp32 on a bf16 model, world 1: the gradient finish()
    returns is the fp32 sum of the micro-steps' bf16 gradients in micro-step order -- bit for bit,
    on the second step too (the accumulator is overwritten by a step's first drain, not zero-filled)."""
    dev = gpu_device()
    _native_lib_loaded()
    from databricks_distributed_deep_learning_amd.optim import ParamArena
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    torch.manual_seed(5)

    def model():
        torch.manual_seed(6)
        return torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 16)).to(dev).bfloat16()

    m, ref = model(), model()
    arena = ParamArena(list(m.named_parameters()))
    ddp = DataParallel(m, arena, bucket_mb=0.01, first_bucket_mb=0.005, accumulate_fp32=True, comm="torch")
    for step in range(2):
        xs = [torch.randn(8, 64, device=dev).bfloat16() for _ in range(3)]
        ys = [torch.randint(0, 16, (8,), device=dev) for _ in range(3)]
        ddp.zero_grad()
        for i in range(3):
            ctx = ddp.no_sync() if i < 2 else torch.enable_grad()
            with ctx:
                torch.nn.functional.cross_entropy(ddp(xs[i]).float(), ys[i]).backward()
        g = ddp.finish().clone()
        # reference: each micro-step's bf16 gradient on its own, summed in fp32 in order
        acc = {}
        for i in range(3):
            ref.zero_grad(set_to_none=True)
            torch.nn.functional.cross_entropy(ref(xs[i]).float(), ys[i]).backward()
            for n, p_ in ref.named_parameters():
                acc[n] = p_.grad.float() if i == 0 else acc[n] + p_.grad.float()
        for e in arena.entries:
            got = g[e.offset:e.offset + e.numel].view(acc[e.name].shape)
            assert torch.equal(got, acc[e.name]), (step, e.name, (got - acc[e.name]).abs().max())
