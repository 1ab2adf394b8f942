"""ZeRO-1 parameter all-gathers vs the forward that reads the parameters (parallel/ddp.py).

With ``shard=True`` each bucket's updated chunks come back through an asynchronous all-gather
and forward pre-hooks wait for exactly the buckets a module's forward reads.  Fused ops read
parameters of modules whose own forward never runs (a bottleneck hands ``bn3`` and
``downsample.bn`` to ``conv_bn_add_bn``, ResNet's root reads the stem, ViT's root the patch
embedding), so a missing wait would let a kernel read a half-written chunk -- silently.

Here the all-gather is "lazy" and poisoned: a fake engine fills every gathered range with NaN
(this rank's own chunk excepted) and writes the real values back only when the range is waited
for.  A forward that reads any parameter before its wait produces NaN.  Runs single-process
on CPU with the world size patched, over world sizes and bucket sizes that put the
boundaries in different places (the advisor's counter-example was world 32, buckets 1-16 MB).
"""
import pytest
import torch

from databricks_distributed_deep_learning_amd.models import BertConfig, BertForSequenceClassification, resnet50
from databricks_distributed_deep_learning_amd.models.vit import ViTConfig, ViTForImageClassification
from databricks_distributed_deep_learning_amd.optim import ParamArena
from databricks_distributed_deep_learning_amd.parallel import dist as ddist
from databricks_distributed_deep_learning_amd.parallel.ddp import DataParallel


class LazyGatherEngine:
    """all_gather poisons the destination and returns a sequence number; ``wait_upto(seq)``
    lands every gather numbered <= seq (the comm stream is in order)."""

    def __init__(self):
        self.seq = 0
        self.pending = {}        # seq -> (recv view, true values)
        self.waited = []

    def all_gather(self, send, recv):
        self.seq += 1
        true = recv.detach().clone()
        with torch.no_grad():
            recv.fill_(float("nan"))
            recv[:send.numel()].copy_(true[:send.numel()])    # rank 0's own chunk is local
        self.pending[self.seq] = (recv, true)
        return self.seq

    def wait_upto(self, seq):
        self.waited.append(seq)
        for s in sorted(k for k in self.pending if k <= seq):
            recv, true = self.pending.pop(s)
            with torch.no_grad():
                recv.copy_(true)

    def wait(self):
        self.wait_upto(self.seq)

    def all_reduce(self, t, average=False):
        return 0

    def reduce_scatter(self, send, recv, average=False):
        return 0


def _tiny_vit():
    c = ViTConfig(image_size=32, patch_size=16, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                  intermediate_size=128, num_labels=10)
    return ViTForImageClassification(c), torch.randn(2, 32, 32, 3)


def _tiny_bert():
    c = BertConfig(vocab_size=101, hidden_size=64, num_hidden_layers=2, num_attention_heads=2, intermediate_size=128,
                   max_position_embeddings=32, num_labels=3, hidden_dropout_prob=0.0,
                   attention_probs_dropout_prob=0.0)
    return BertForSequenceClassification(c), torch.randint(0, 101, (2, 16))


def _resnet():
    return resnet50(num_classes=10), torch.randn(2, 64, 64, 3)


def _forward(model, x):
    if isinstance(model, BertForSequenceClassification):
        return model(x)[0] if isinstance(model(x), tuple) else model(x)
    return model(x)


@pytest.mark.parametrize("world", [2, 8, 32])
@pytest.mark.parametrize("bucket_mb", [0.05, 1.0, 4.0])
@pytest.mark.parametrize("build", [_resnet, _tiny_bert, _tiny_vit], ids=["resnet50", "bert", "vit"])
def test_every_parameter_waited_before_use(monkeypatch, world, bucket_mb, build):
    monkeypatch.setattr(ddist, "world_size", lambda: world)
    torch.manual_seed(0)
    model, x = build()
    model.eval()
    with torch.no_grad():
        ref = model(x)
    ref = ref[0] if isinstance(ref, tuple) else ref
    arena = ParamArena(list(model.named_parameters()), pad_multiple=world * 64)
    eng = LazyGatherEngine()
    dp = DataParallel(model, arena, bucket_mb=bucket_mb, first_bucket_mb=bucket_mb / 4, comm=eng, shard=True,
                      broadcast_init=False)
    assert dp.shard and len(dp.buckets) >= 1
    groups = dp.shard_groups()
    ranges = [(a, a + (b - a) // world, None) for a, b in groups]
    dp.gather_params(groups, ranges)
    assert torch.isnan(arena.flat).any()             # the poison is in place before the forward
    with torch.no_grad():
        out = dp(x)
    out = out[0] if isinstance(out, tuple) else out
    assert torch.isfinite(out).all(), "a parameter was read before its bucket's all-gather was waited for"
    torch.testing.assert_close(out, ref)
    dp.close()


def test_gather_waits_stay_overlapped(monkeypatch):
    """The root waits only for what its own forward reads: a BERT forward starts with most of
    the encoder's all-gathers still in flight (waited for layer by layer)."""
    monkeypatch.setattr(ddist, "world_size", lambda: 2)
    torch.manual_seed(0)
    model, x = _tiny_bert()
    model.eval()
    arena = ParamArena(list(model.named_parameters()), pad_multiple=128)
    eng = LazyGatherEngine()
    dp = DataParallel(model, arena, bucket_mb=0.02, first_bucket_mb=0.01, comm=eng, shard=True,
                      broadcast_init=False)
    seen = []
    h = model.bert.layers[0].register_forward_pre_hook(lambda *_: seen.append(len(eng.pending)))
    groups = dp.shard_groups()
    dp.gather_params(groups, [(a, a + (b - a) // 2, None) for a, b in groups])
    n = len(eng.pending)
    with torch.no_grad():
        dp(x)
    h.remove()
    assert n >= 4 and seen and seen[0] > 0, (n, seen)
    dp.close()
