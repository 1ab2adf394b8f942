"""Native step glue (csrc/kernels/elementwise.hip, ops/glue.py) against plain PyTorch fp32 / int64
references: the kernels that replaced the ATen launches of the BERT step."""
import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 7, 1000, 2048, 4096, 8192, 16384, 16385, 32768])
def test_sort_ids_is_the_stable_sort(n):
    """The one-workgroup bitonic sort of (id, position) keys == torch's stable sort (ids and the
    permutation), with long runs of one id (padding) and two-valued ids (token types)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops._lib import call, fn, p
    torch.manual_seed(n)
    for V, ids in [(30522, torch.randint(0, 30522, (n,), device=dev)),
                   (30522, torch.where(torch.rand(n, device=dev) < 0.6, 0, torch.randint(0, 30522, (n,), device=dev))),
                   (2, torch.randint(0, 2, (n,), device=dev))]:
        assert fn("ddl_sort_ids_ok")(n, V) == 1
        s = torch.empty(n, dtype=torch.int32, device=dev)
        pi = torch.empty(n, dtype=torch.int64, device=dev)
        call("ddl_sort_ids", p(ids), n, p(s), p(pi))
        ws, wpi = torch.sort(ids, stable=True)
        assert torch.equal(s.long(), ws) and torch.equal(pi, wpi)
    assert fn("ddl_sort_ids_ok")(32769, 100) == 0 and fn("ddl_sort_ids_ok")(16384, 1 << 19) == 0


def test_copy2d_pad_slice_gather_and_zero():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_elementwise as E
    torch.manual_seed(0)
    for dt in (torch.bfloat16, torch.float32):
        w = torch.randn(2, 768, device=dev).to(dt)
        wp = E.copy2d(torch.full((8, 768), 7.0, device=dev).to(dt), w, 768, 8, 768, 768, 2, 768)
        assert torch.equal(wp[:2], w) and not wp[2:].any()
        y = torch.randn(100, 8, device=dev).to(dt)
        out = E.copy2d(torch.empty(100, 2, device=dev).to(dt), y, 2, 100, 2, 8, 100, 2)
        assert torch.equal(out, y[:, :2])
        dyp = E.copy2d(torch.full((100, 8), 3.0, device=dev).to(dt), out, 8, 100, 8, 2, 100, 2)
        assert torch.equal(dyp[:, :2], out) and not dyp[:, 2:].any()
        h = torch.randn(4, 128, 768, device=dev).to(dt)
        first = E.copy2d(torch.empty(4, 768, device=dev).to(dt), h, 768, 4, 768, 128 * 768, 4, 768)
        assert torch.equal(first, h[:, 0])
        b = torch.randn(6, device=dev).to(dt)
        bp = E.copy2d(torch.full((8,), 1.0, device=dev).to(dt), b, 8, 1, 8, 6, 1, 6)
        assert torch.equal(bp[:6], b) and not bp[6:].any()
        z = torch.randn(1000003, device=dev).to(dt) + 5.0
        E.zero_(z[1:])                                   # unaligned start and odd length
        assert z[0] != 0 and not z[1:].any()
        z2 = torch.randn(12345, device=dev).to(dt)
        E.zero_(z2)
        assert not z2.any()


def test_tanh_bwd_and_add_into():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_elementwise as E
    torch.manual_seed(1)
    for n in (128 * 768, 13):
        y = torch.tanh(torch.randn(n, device=dev)).bfloat16()
        dy = torch.randn(n, device=dev).bfloat16()
        ref = dy.float() * (1 - y.float() ** 2)
        torch.testing.assert_close(E.tanh_bwd(dy, y).float(), ref, rtol=1e-2, atol=1e-2)
        a = torch.randn(n, device=dev).bfloat16()
        before = a.float().clone()
        E.add_into(a, dy)
        torch.testing.assert_close(a.float(), (before + dy.float()).bfloat16().float(), rtol=0, atol=0)


def test_first_token_and_embedding_residual_autograd():
    """ops.first_token / ops.embedding_residual: values and gradients equal to the PyTorch
    expressions they replace, with and without gradient-arena sinks."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(2)
    h = torch.randn(4, 128, 768, device=dev).bfloat16().requires_grad_()
    g = torch.randn(4, 768, device=dev).bfloat16()
    out = ops.first_token(h)
    out.backward(g)
    h2 = h.detach().clone().requires_grad_()
    h2[:, 0].contiguous().backward(g)
    assert torch.equal(out, h.detach()[:, 0]) and torch.equal(h.grad, h2.grad)

    pos = torch.randn(512, 768, device=dev).bfloat16().requires_grad_()
    tok = torch.randn(2, 768, device=dev).bfloat16().requires_grad_()
    r = ops.embedding_residual(pos, tok, 128)
    ref_p, ref_t = pos.detach().clone().requires_grad_(), tok.detach().clone().requires_grad_()
    ref = ref_p[:128].unsqueeze(0) + ref_t[0].view(1, 1, -1)
    assert torch.equal(r, ref)
    dr = torch.randn(1, 128, 768, device=dev).bfloat16()
    r.backward(dr)
    ref.backward(dr)
    assert torch.equal(pos.grad, ref_p.grad)
    torch.testing.assert_close(tok.grad.float(), ref_t.grad.float(), rtol=1e-2, atol=5e-2)
    # arena sinks: the gradient lands in the slots (accumulated), autograd gets None
    pos2 = torch.nn.Parameter(pos.detach().clone())
    tok2 = torch.nn.Parameter(tok.detach().clone())
    sp, st = torch.ones(512, 768, device=dev).bfloat16(), torch.ones(2, 768, device=dev).bfloat16()
    ready = []
    pos2._ddl_main_grad, tok2._ddl_main_grad = sp, st
    pos2._ddl_grad_ready = lambda: ready.append("pos")
    tok2._ddl_grad_ready = lambda: ready.append("tok")
    ops.embedding_residual(pos2, tok2, 128).backward(dr)
    assert sorted(ready) == ["pos", "tok"] and pos2.grad is None and tok2.grad is None
    torch.testing.assert_close(sp[:128].float(), (1 + dr[0].float()).bfloat16().float(), rtol=0, atol=0)
    assert torch.equal(sp[128:], torch.ones_like(sp[128:]))
    torch.testing.assert_close(st[0].float(), 1 + dr[0].float().sum(0), rtol=1e-2, atol=0.3)
    assert torch.equal(st[1], torch.ones_like(st[1]))


@pytest.mark.parametrize("dt,B,P,H", [(torch.bfloat16, 16, 196, 768), (torch.bfloat16, 3, 5, 24),
                                      (torch.float32, 4, 49, 64), (torch.bfloat16, 2, 7, 20)])
def test_prepend_token_add_autograd(dt, B, P, H):
    """ops.prepend_token_add (ViT's [cls | patches] + position embeddings, ddl_seq_prepend_add): values
    equal to the cat + add it replaces; gradients against the fp32 reference, with and without
    gradient-arena sinks (H = 20: the scalar kernel path)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(3)
    x = torch.randn(B, P, H, device=dev).to(dt).requires_grad_()
    cls = torch.randn(1, 1, H, device=dev).to(dt).requires_grad_()
    pos = torch.randn(1, P + 1, H, device=dev).to(dt).requires_grad_()
    out = ops.prepend_token_add(x, cls, pos)
    ref = torch.cat([cls.detach().expand(B, -1, -1), x.detach()], 1) + pos.detach()
    assert out.shape == (B, P + 1, H) and torch.equal(out, ref)
    g = torch.randn(B, P + 1, H, device=dev).to(dt)
    out.backward(g)
    gf = g.float()
    assert torch.equal(x.grad, g[:, 1:])
    torch.testing.assert_close(pos.grad.float(), gf.sum(0, keepdim=True), rtol=1e-2, atol=0.1)
    torch.testing.assert_close(cls.grad.float(), gf[:, :1].sum(0, keepdim=True), rtol=1e-2, atol=0.1)
    # arena sinks: both parameter gradients accumulate into their slots, autograd gets None
    cls2, pos2 = torch.nn.Parameter(cls.detach().clone()), torch.nn.Parameter(pos.detach().clone())
    sc, sp = torch.ones(1, 1, H, device=dev).to(dt), torch.ones(1, P + 1, H, device=dev).to(dt)
    ready = []
    cls2._ddl_main_grad, pos2._ddl_main_grad = sc, sp
    cls2._ddl_grad_ready = lambda: ready.append("cls")
    pos2._ddl_grad_ready = lambda: ready.append("pos")
    ops.prepend_token_add(x.detach(), cls2, pos2).backward(g)
    assert sorted(ready) == ["cls", "pos"] and cls2.grad is None and pos2.grad is None
    torch.testing.assert_close(sp.float(), 1 + gf.sum(0, keepdim=True), rtol=1e-2, atol=0.2)
    torch.testing.assert_close(sc.float(), 1 + gf[:, :1].sum(0, keepdim=True), rtol=1e-2, atol=0.2)


def test_classifier_head_padded_linear_matches_reference():
    """_LinearPadN (N = 2 classes, padded to 8 rows): forward, dx, dW, db against fp32 PyTorch, twice
    (the padded W is cached per parameter version and rebuilt after an in-place update)."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(3)
    x = torch.randn(128, 768, device=dev).bfloat16().requires_grad_()
    w = torch.nn.Parameter((torch.randn(2, 768, device=dev) * 0.02).bfloat16())
    b = torch.nn.Parameter(torch.randn(2, device=dev).bfloat16())
    for it in range(2):
        x.grad = w.grad = b.grad = None
        y = ops.linear(x, w, b, None)
        dy = torch.randn(128, 2, device=dev).bfloat16()
        y.backward(dy)
        ref = x.detach().float() @ w.detach().float().t() + b.detach().float()
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(x.grad.float(), dy.float() @ w.detach().float(), rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(w.grad.float(), dy.float().t() @ x.detach().float(), rtol=2e-2, atol=0.1)
        torch.testing.assert_close(b.grad.float(), dy.float().sum(0), rtol=2e-2, atol=0.1)
        with torch.no_grad():
            w.mul_(-1.5)                      # version bump: the padded copy must be rebuilt


@pytest.mark.parametrize("H,W,C,pad", [(224, 224, 3, 3), (31, 29, 3, 3), (16, 16, 4, 1), (15, 17, 1, 2)])
def test_stem_space_to_depth_transforms_native(H, W, C, pad):
    """ddl_s2d_input / ddl_s2d_weight (one native pass each) == the pad + permute reference (the same
    functions on CPU tensors), odd extents included."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
    torch.manual_seed(H + W)
    x = torch.randn(2, H, W, C).bfloat16()
    w = torch.randn(64, 7, 7, C).bfloat16()
    assert torch.equal(NC._s2d_input(x.to(dev), pad).cpu(), NC._s2d_input(x, pad))
    assert torch.equal(NC._s2d_weight(w.to(dev)).cpu(), NC._s2d_weight(w))
