"""Model-zoo tests on CPU: parameter counts and HF parity."""
import pytest
import torch

from databricks_distributed_deep_learning_amd import models as M


@pytest.mark.parametrize("name,n,classes", [
    ("resnet18", 11_689_512, 1000),
    ("resnet50", 25_557_032, 1000),
    ("bert_base", 109_483_778, 2),
    ("bert_large", 335_143_938, 2),
    ("vit_b16", 86_567_656, 1000),
])
def test_param_counts(name, n, classes):
    assert M.count_params(M.build_model(name, num_classes=classes)) == n


def test_resnet_forward_backward_shapes():
    m = M.resnet18(num_classes=10)
    x = torch.randn(2, 64, 64, 3, requires_grad=True)
    y = m(x)
    assert y.shape == (2, 10)
    y.sum().backward()
    assert x.grad.shape == x.shape
    assert all(p.grad is not None for p in m.parameters())


def test_resnet50_matches_torchvision_style_nchw_reference():
    """Our NHWC ResNet-50 equals an NCHW functional re-implementation (weights shared)."""
    import torch.nn.functional as F
    torch.manual_seed(0)
    m = M.resnet50(num_classes=7).eval()
    for mod in m.modules():  # non-trivial BN statistics
        if hasattr(mod, "running_mean"):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 1.5)
    x = torch.randn(1, 3, 64, 64)
    sd = m.state_dict()

    def conv(t, name, s, p):
        return F.conv2d(t, sd[name].permute(0, 3, 1, 2), stride=s, padding=p)

    def bn(t, name):
        return F.batch_norm(t, sd[name + ".running_mean"], sd[name + ".running_var"], sd[name + ".weight"],
                            sd[name + ".bias"], False, 0.0, 1e-5)
    h = F.relu(bn(conv(x, "conv1.weight", 2, 3), "bn1"))
    h = F.max_pool2d(h, 3, 2, 1)
    for li, (blocks, stride) in enumerate(zip([3, 4, 6, 3], [1, 2, 2, 2]), 1):
        for bi in range(blocks):
            pre = f"layer{li}.{bi}."
            s = stride if bi == 0 else 1
            idt = h
            if pre + "downsample.0.weight" in sd:
                idt = bn(conv(h, pre + "downsample.0.weight", s, 0), pre + "downsample.1")
            o = F.relu(bn(conv(h, pre + "conv1.weight", 1, 0), pre + "bn1"))
            o = F.relu(bn(conv(o, pre + "conv2.weight", s, 1), pre + "bn2"))
            h = F.relu(bn(conv(o, pre + "conv3.weight", 1, 0), pre + "bn3") + idt)
    ref = F.linear(h.mean((2, 3)), sd["fc.weight"], sd["fc.bias"])
    ours = m(x.permute(0, 2, 3, 1).contiguous())
    torch.testing.assert_close(ours, ref, atol=1e-4, rtol=1e-4)


def test_bert_matches_hf_random_init():
    transformers = pytest.importorskip("transformers")
    from databricks_distributed_deep_learning_amd.models.bert import BertConfig, BertForSequenceClassification, \
        from_hf_state_dict, to_hf_state_dict
    hc = transformers.BertConfig(vocab_size=100, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                 intermediate_size=128, max_position_embeddings=32, num_labels=3,
                                 hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    hf = transformers.BertForSequenceClassification(hc).eval()
    ours = BertForSequenceClassification(BertConfig(vocab_size=100, hidden_size=64, num_hidden_layers=2,
                                                    num_attention_heads=4, intermediate_size=128,
                                                    max_position_embeddings=32, num_labels=3,
                                                    hidden_dropout_prob=0.0,
                                                    attention_probs_dropout_prob=0.0)).eval()
    missing, unexpected = ours.load_state_dict(from_hf_state_dict(hf.state_dict(), 2), strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    ids = torch.randint(0, 100, (2, 11))
    mask = torch.ones(2, 11, dtype=torch.long)
    mask[1, 8:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask).logits
        got = ours(ids, mask)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)
    back = to_hf_state_dict(ours.state_dict(), 2)
    for k, v in back.items():
        torch.testing.assert_close(v, hf.state_dict()[k])


def test_vit_matches_hf_random_init():
    transformers = pytest.importorskip("transformers")
    from databricks_distributed_deep_learning_amd.models.vit import ViTConfig, ViTForImageClassification, \
        from_hf_state_dict
    hc = transformers.ViTConfig(image_size=32, patch_size=16, hidden_size=64, num_hidden_layers=2,
                                num_attention_heads=4, intermediate_size=128, num_labels=5)
    torch.manual_seed(0)
    hf = transformers.ViTForImageClassification(hc).eval()
    ours = ViTForImageClassification(ViTConfig(image_size=32, patch_size=16, hidden_size=64, num_hidden_layers=2,
                                               num_attention_heads=4, intermediate_size=128,
                                               num_labels=5)).eval()
    ours.load_state_dict(from_hf_state_dict(hf.state_dict(), 2))
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        ref = hf(pixel_values=x).logits
        got = ours(x.permute(0, 2, 3, 1).contiguous())
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


def test_cast_params_keeps_bn_stats_fp32():
    m = M.resnet18()
    M.cast_params(m, torch.bfloat16)
    assert all(p.dtype == torch.bfloat16 for p in m.parameters())
    assert m.bn1.running_mean.dtype == torch.float32


def test_grad_bridge_offer_either_order():
    """GradBridge.offer/take: a sibling producer's gradient is summed exactly once
    whether the consumer runs after it (offer accepted) or before it (offer refused)."""
    from databricks_distributed_deep_learning_amd.ops.bridge import GradBridge
    g_prod, g_cons = torch.full((3,), 2.0), torch.full((3,), 5.0)
    b = GradBridge()                      # producer first
    assert b.offer(g_prod)
    r = b.take()
    total = g_cons + r
    assert torch.equal(total, torch.full((3,), 7.0))
    b = GradBridge()                      # consumer first: nothing pending, bridge closes
    assert b.take() is None
    assert not b.offer(g_prod)            # producer keeps its gradient for autograd
    assert b.grad is None
