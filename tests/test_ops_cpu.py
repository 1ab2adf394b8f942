"""CPU unit tests of the op layer (SURVEY §4.2 "Unit: ops/autograd").

* ``torch.autograd.gradcheck`` of the reference ops the native kernels are measured
  against (NHWC conv, Linear + activations, LayerNorm + residual, BatchNorm training,
  attention with a key mask, pools, cross-entropy) -- the oracles must have correct
  gradients before a GPU test can trust them.  Ops that compute in fp32 internally are
  checked in fp32 with finite-difference tolerances to match;
* the residual-gradient bridge (``ops.bridge.GradBridge``): put / offer / take
  semantics and the reference-path join, which must sum the bridged gradient exactly once;
* the pre-LN wiring (``linear(residual_grad_to=)`` + ``layer_norm(grad_from=)``) on the
  reference path equals plain autograd.
"""
import importlib

import pytest
import torch

from databricks_distributed_deep_learning_amd import ops
from databricks_distributed_deep_learning_amd.ops.bridge import GradBridge, join

# the op submodules (``ops`` re-exports same-named functions, so import them by path)
A, CV, LI, NO, PO = (importlib.import_module(f"databricks_distributed_deep_learning_amd.ops.{m}")
                     for m in ("attention", "conv", "linear", "norm", "pool"))

F32 = dict(eps=1e-3, atol=2e-2, rtol=2e-2)
# (fp32 gradchecks are deliberate: the oracles compute in fp32 whatever the input dtype)
pytestmark = pytest.mark.filterwarnings("ignore:Input #.*double precision:UserWarning")


def _r(*shape, dtype=torch.float64, scale=1.0):
    return (torch.randn(*shape, dtype=dtype) * scale).requires_grad_(True)


@pytest.mark.parametrize("stride,pad,k", [(1, 1, 3), (2, 1, 3), (2, 0, 1)])
def test_gradcheck_conv2d_nhwc(stride, pad, k):
    torch.manual_seed(0)
    x, w = _r(2, 7, 6, 3), _r(4, k, k, 3, scale=0.3)
    assert torch.autograd.gradcheck(lambda a, b: CV.conv2d_reference(a, b, stride, pad), (x, w))


@pytest.mark.parametrize("act", [None, "gelu", "tanh"])
def test_gradcheck_linear_act(act):
    torch.manual_seed(1)
    x, w, b = _r(5, 6, dtype=torch.float32), _r(4, 6, dtype=torch.float32, scale=0.3), _r(4, dtype=torch.float32)
    assert torch.autograd.gradcheck(lambda a, ww, bb: LI.linear_reference(a, ww, bb, act), (x, w, b), **F32)


def test_gradcheck_layer_norm_residual():
    torch.manual_seed(2)
    x, r = _r(3, 8, dtype=torch.float32), _r(3, 8, dtype=torch.float32)
    g, b = _r(8, dtype=torch.float32), _r(8, dtype=torch.float32)
    assert torch.autograd.gradcheck(lambda a, rr, gg, bb: NO.layer_norm_reference(a, gg, bb, 1e-5, rr),
                                    (x, r, g, b), **F32)


def test_gradcheck_batch_norm_train_residual():
    torch.manual_seed(3)
    x, r = _r(4, 3, 3, 5, dtype=torch.float32), _r(4, 3, 3, 5, dtype=torch.float32)
    g, b = _r(5, dtype=torch.float32), _r(5, dtype=torch.float32)

    def f(a, rr, gg, bb):
        rm, rv = torch.zeros(5), torch.ones(5)
        return NO.batch_norm_reference(a, gg, bb, rm, rv, True, 0.1, 1e-5, False, rr)
    assert torch.autograd.gradcheck(f, (x, r, g, b), **F32)


def test_gradcheck_attention_masked():
    torch.manual_seed(4)
    B, S, H, D = 2, 5, 2, 4
    qkv = _r(B, S, 3 * H * D, dtype=torch.float32, scale=0.5)
    mask = torch.zeros(B, S)
    mask[1, 3:] = -10000.0
    assert torch.autograd.gradcheck(lambda t: A.attention_reference(t, H, mask), (qkv,), **F32)


def test_gradcheck_pools_and_loss():
    torch.manual_seed(5)
    x = _r(2, 6, 6, 3)
    assert torch.autograd.gradcheck(lambda a: PO.max_pool2d_reference(a, 3, 2, 1), (x,))
    logits = _r(4, 7, dtype=torch.float32)
    labels = torch.randint(0, 7, (4,))
    assert torch.autograd.gradcheck(lambda z: ops.cross_entropy(z, labels), (logits,), **F32)


def test_grad_bridge_semantics():
    b = GradBridge()
    g = torch.ones(3)
    b.put(g)
    with pytest.raises(RuntimeError):
        b.put(g)                          # a second pending gradient: the bridge was reused
    assert b.take() is g and b.take() is None
    assert not b.offer(g)                 # the consumer already ran: the producer keeps it
    b2 = GradBridge()
    assert b2.offer(g) and b2.take() is g


def test_bridge_join_sums_once():
    """Reference-path join: identity forward, the bridged gradient added once in backward."""
    x = torch.randn(4, requires_grad=True)
    br = GradBridge()
    y = join(x, br) * 2.0
    br.put(torch.full((4,), 10.0))
    y.sum().backward()
    assert torch.equal(x.grad, torch.full((4,), 12.0))
    x.grad = None
    y = join(x, GradBridge()) * 2.0       # empty bridge: nothing added
    y.sum().backward()
    assert torch.equal(x.grad, torch.full((4,), 2.0))


def test_pre_ln_residual_bridge_reference_path():
    """ViT block wiring on the reference ops: the residual branch's gradient reaches h once
    (through autograd on this path; the native path hands it to the LayerNorm backward)."""
    torch.manual_seed(6)
    H = 8
    h = torch.randn(3, H, requires_grad=True)
    w, bw = torch.randn(H, H) * 0.3, torch.randn(H)
    g, bb = torch.rand(H) + 0.5, torch.randn(H)

    def block(bridged):
        br = GradBridge() if bridged else None
        y = ops.layer_norm(h, g, bb, 1e-5, grad_from=br)
        return ops.linear(y, w, bw, residual=h, residual_grad_to=br)

    grads = []
    for bridged in (True, False):
        h.grad = None
        block(bridged).square().sum().backward()
        grads.append(h.grad.clone())
    ref = h.detach().clone().requires_grad_(True)
    out = torch.nn.functional.linear(torch.nn.functional.layer_norm(ref, (H,), g, bb, 1e-5), w, bw) + ref
    out.square().sum().backward()
    torch.testing.assert_close(grads[0], grads[1])
    torch.testing.assert_close(grads[0], ref.grad, rtol=1e-4, atol=1e-5)
