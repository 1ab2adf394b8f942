"""Whole-model numerics on the GPU: the native bf16 path (HIP kernels, fused
BN/residual/bridged residual gradients, flash attention, fused linears) against
the stock-PyTorch fp32 path (``native=off``) on the same weights and inputs.

A randomly initialised deep net is badly conditioned: stock PyTorch in bf16 is
itself 30-60 % (max-abs relative) away from fp32 on many gradients.  So the
criterion is "as accurate as stock bf16": for every parameter the native
error against fp32 must stay within a small factor of stock-bf16's error, and
the mean over all parameters within 25 %.  A broken backward kernel (wrong
tap, dropped residual gradient, transposed write) is far outside that band.
"""
import copy

import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-8)).item()


def _grads(model, run, native: str):
    from databricks_distributed_deep_learning_amd import ops
    ops.set_native_mode(native)
    try:
        model.zero_grad(set_to_none=True)
        loss = run(model)
        loss.backward()
        torch.cuda.synchronize()
        return loss.detach().float(), {n: p.grad.detach().float().clone() for n, p in model.named_parameters()
                                      if p.grad is not None}
    finally:
        ops.set_native_mode("auto")


def _compare(model_fp32, run, names, tol=None):
    from databricks_distributed_deep_learning_amd.models.layers import cast_params
    ref_loss, ref = _grads(model_fp32, run, "off")
    m_t = cast_params(copy.deepcopy(model_fp32), torch.bfloat16)
    t_loss, t16 = _grads(m_t, run, "off")
    m16 = cast_params(copy.deepcopy(model_fp32), torch.bfloat16)
    loss, got = _grads(m16, run, "auto")
    # random-init deep nets amplify rounding chaotically (layer outputs drift 10-20 % by
    # ResNet-50's layer3 in stock bf16 too); the per-parameter band below is the real check
    assert abs(loss.item() - ref_loss.item()) <= 3 * abs(t_loss.item() - ref_loss.item()) + \
        5e-2 * max(1.0, abs(ref_loss.item())), (loss, t_loss, ref_loss)
    # nothing may silently lose its gradient (e.g. a bridged residual that was never consumed)
    assert set(got) == set(ref)
    e_nat = {n: _rel(got[n], ref[n]) for n in ref}
    e_t16 = {n: _rel(t16[n], ref[n]) for n in ref}
    for n in names:
        assert n in got, f"no gradient for {n} on the native path"
    bad = {n: (round(e_nat[n], 3), round(e_t16[n], 3)) for n in ref if e_nat[n] > 2.0 * e_t16[n] + 0.05}
    assert not bad, bad
    mean_nat = sum(e_nat.values()) / len(e_nat)
    mean_t16 = sum(e_t16.values()) / len(e_t16)
    assert mean_nat <= 1.25 * mean_t16 + 0.02, (mean_nat, mean_t16)
    return len(names)


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_resnet_native_vs_reference(arch):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import models
    torch.manual_seed(0)
    m = getattr(models, arch)(num_classes=10).to(dev).train()
    x = torch.randn(8, 96, 96, 3, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)

    def run(mod):
        from databricks_distributed_deep_learning_amd import ops
        xin = x.to(next(mod.parameters()).dtype)
        return ops.cross_entropy(mod(xin).float(), y)

    names = ["conv1.weight", "bn1.weight", "layer1.0.conv1.weight", "layer1.1.conv1.weight",
             "layer2.1.conv1.weight", "layer3.0.downsample.0.weight", "layer4.1.bn2.bias", "fc.weight", "fc.bias"]
    assert _compare(m, run, names) == len(names)


def test_bert_native_vs_reference():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.models.bert import BertConfig, BertForSequenceClassification
    torch.manual_seed(0)
    cfg = BertConfig(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertForSequenceClassification(cfg).to(dev).train()
    ids = torch.randint(0, cfg.vocab_size, (4, 128), device=dev)
    mask = torch.ones(4, 128, device=dev)
    mask[1, 100:] = 0
    labels = torch.randint(0, 2, (4,), device=dev)

    def run(mod):
        loss, _ = mod(ids, mask, labels=labels)
        return loss.float()

    names = ["bert.embeddings.word_embeddings.weight", "bert.layers.0.qkv.weight", "bert.layers.0.qkv.bias",
             "bert.layers.1.ffn_in.weight", "bert.layers.1.ffn_out.bias", "bert.layers.1.ffn_ln.weight",
             "classifier.weight"]
    names = [n for n in names if n in dict(m.named_parameters())]
    assert len(names) >= 4
    _compare(m, run, names)


def test_vit_native_vs_reference():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.models.vit import ViTConfig, ViTForImageClassification
    torch.manual_seed(0)
    m = ViTForImageClassification(ViTConfig(image_size=64, num_hidden_layers=2, num_labels=10)).to(dev).train()
    x = torch.randn(4, 64, 64, 3, device=dev)
    y = torch.randint(0, 10, (4,), device=dev)

    def run(mod):
        from databricks_distributed_deep_learning_amd import ops
        return ops.cross_entropy(mod(x.to(next(mod.parameters()).dtype)).float(), y)

    names = [n for n, _ in m.named_parameters()][:3] + [n for n, _ in m.named_parameters()][-3:]
    _compare(m, run, names)


def test_vit_layernorm_grad_bridge_matches_autograd_sum():
    """Pre-LN residual-stream gradient added inside the LayerNorm backward (ViT: the output
    Linear hands its residual gradient over, ln_bwd_k<ADD>) equals autograd's separate add
    -- including the fc2 / attn_out bias gradients, which come from the LN's column sums."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.models import vit as V
    from databricks_distributed_deep_learning_amd.models.layers import cast_params
    torch.manual_seed(0)
    m = cast_params(V.ViTForImageClassification(V.ViTConfig(image_size=64, num_hidden_layers=3, num_labels=10)),
                    torch.bfloat16).to(dev).train()
    x = torch.randn(4, 64, 64, 3, device=dev, dtype=torch.bfloat16)
    y = torch.randint(0, 10, (4,), device=dev)

    def run(mod):
        from databricks_distributed_deep_learning_amd import ops
        return ops.cross_entropy(mod(x).float(), y)

    out = {}
    for flag in (True, False):
        V._LN_BRIDGE = flag
        try:
            out[flag] = _grads(copy.deepcopy(m), run, "auto")[1]
        finally:
            V._LN_BRIDGE = True
    assert set(out[True]) == set(out[False])
    for n in out[True]:
        assert _rel(out[True][n], out[False][n]) < 2e-2, n


def test_residual_grad_bridge_matches_autograd_sum():
    """Identity-block residual gradient fused into conv1's dgrad epilogue (ops/bridge.py)
    equals autograd's separate add, up to one bf16 rounding."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import models
    from databricks_distributed_deep_learning_amd.models import resnet as R
    from databricks_distributed_deep_learning_amd.models.layers import cast_params
    torch.manual_seed(0)
    m = cast_params(models.resnet50(num_classes=10), torch.bfloat16).to(dev).train()
    x = torch.randn(8, 64, 64, 3, device=dev, dtype=torch.bfloat16)
    y = torch.randint(0, 10, (8,), device=dev)

    def run(mod):
        from databricks_distributed_deep_learning_amd import ops
        return ops.cross_entropy(mod(x).float(), y)

    out = {}
    for flag in (True, False):
        R._BRIDGE = flag
        try:
            mm = copy.deepcopy(m)
            out[flag] = _grads(mm, run, "auto")[1]
        finally:
            R._BRIDGE = True
    # the deep end of the net amplifies one extra bf16 rounding per block (random init is
    # ill-conditioned), so the tight check covers the parameters near the bridged blocks
    near = [n for n in out[True] if n.startswith(("layer3.", "layer4.", "fc."))]
    assert len(near) > 30
    for n in near:
        assert _rel(out[True][n], out[False][n]) < 3e-2, n
    for n in out[True]:
        assert _rel(out[True][n], out[False][n]) < 0.15, n


@pytest.mark.parametrize("kind,stride", [("bottleneck", 1), ("bottleneck", 2), ("basic", 2)])
def test_downsample_sibling_bridge(kind, stride):
    """Downsample blocks: conv1 offers its input gradient to the downsample conv, whose
    dgrad epilogue adds it (in place over the strided parity class for stride 2); the
    block input's gradient equals autograd's separate sum."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.models import resnet as R
    from databricks_distributed_deep_learning_amd.models.layers import cast_params
    torch.manual_seed(3)
    cin, planes = 64, 32
    if kind == "bottleneck":
        blk = R.Bottleneck(cin, planes, stride, R.Downsample(cin, planes * 4, stride))
    else:
        blk = R.BasicBlock(cin, planes, stride, R.Downsample(cin, planes, stride))
    blk = cast_params(blk, torch.bfloat16).to(dev).train()
    x0 = torch.randn(4, 20, 20, cin, device=dev, dtype=torch.bfloat16)
    grads = {}
    for flag in (True, False):
        R._BRIDGE = flag
        try:
            b = copy.deepcopy(blk)
            x = x0.clone().requires_grad_(True)
            y = b(x)
            y.backward(torch.ones_like(y) * 0.01 + (y.detach() * 0.1))
            grads[flag] = x.grad.float()
        finally:
            R._BRIDGE = True
    assert _rel(grads[True], grads[False]) < 1e-2


@pytest.mark.parametrize("preset,over", [
    ("resnet50_ddp", dict(model="resnet18", batch_size=16, image_size=64, num_classes=10)),
    ("bert_base_ddp", dict(batch_size=8, seq_len=64)),
])
def test_side_stream_weight_gradients_match(preset, over, monkeypatch):
    """Weight-gradient GEMMs on the side stream (concurrent with the same layer's dgrad,
    _lib.side_stream) give bit-identical training to the single-stream order."""
    gpu_device()
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.ops import _lib, _native_gemm
    # in-model tuning would run the first trainer's warm-up on rotating candidates and the second
    # one's on the committed plan: pin the isolated tuner so both take the same kernels
    monkeypatch.setattr(_native_gemm, "_ONLINE_ENV", "0")
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    finals = []
    prev = _lib.wgrad_stream_enabled()
    try:
        for on in (False, True):
            _lib.set_wgrad_stream(on)
            t = Trainer(get_preset(preset, steps=3, warmup_steps=1, log_every=0, **over))
            t.run()
            torch.cuda.synchronize()
            finals.append(t.arena.flat.float().clone())
            del t
    finally:
        _lib.set_wgrad_stream(prev)
    assert torch.equal(finals[0], finals[1]), (finals[0] - finals[1]).abs().max()
