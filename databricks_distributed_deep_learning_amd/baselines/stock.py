"""Stock PyTorch-ROCm arm of the benchmark (BASELINE.md "What this repo will report
instead", arm (a)).

The reference's own PyTorch path is a plain eager module call
(``/root/reference/notebooks/cv/onnx_experiments.py:173-174``).  This module is the
training equivalent a user of stock PyTorch-ROCm would write, with NONE of this
framework's kernels, arenas or reducers in the loop:

* ResNet-50: ``nn.Conv2d`` / ``nn.BatchNorm2d`` / ``nn.ReLU`` / ``nn.MaxPool2d``
  (MIOpen), channels_last memory format, fp32 parameters under
  ``torch.autocast(bfloat16)``, ``torch.optim.SGD(momentum, fused=True)``;
* BERT-base: ``nn.Linear`` (hipBLASLt), ``F.scaled_dot_product_attention``,
  ``nn.LayerNorm``, ``nn.GELU``, ``nn.Dropout``, same autocast,
  ``torch.optim.AdamW(fused=True)``;
* ViT-B/16: a strided ``nn.Conv2d`` patch embedding, pre-LN encoder layers on the same
  ``nn.Linear`` / SDPA / ``nn.LayerNorm`` / ``nn.GELU`` blocks, ``torch.optim.AdamW(fused=True)``;
* BERT-large (seq 512, grad accumulation under ``DDP.no_sync``): the BERT-base modules at
  hidden 1024 / 24 layers / 16 heads; LAMB, which stock PyTorch does not ship, written with the
  ``torch._foreach_*`` multi-tensor ops a stock user would use (no fused kernel of this framework);
* all wrapped in ``torch.nn.parallel.DistributedDataParallel`` (RCCL buckets,
  overlapped with backward: torch's own reducer), same per-GPU batch and the same
  synthetic device-resident data as the native arm.

Timing follows the bench contract: warm-up steps untimed, then exactly ``steps``
optimizer steps between barrier + device synchronisation, max over ranks.
"""
from __future__ import annotations

import contextlib
import math
import time
from typing import Any, Dict

import torch
import torch.nn as nn
import torch.nn.functional as F


# ---------------------------------------------------------------- ResNet-50 (torchvision-equivalent)
class _Bottleneck(nn.Module):
    def __init__(self, cin: int, planes: int, stride: int, down: bool):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = nn.Sequential(nn.Conv2d(cin, planes * 4, 1, stride, bias=False),
                                        nn.BatchNorm2d(planes * 4)) if down else None

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class StockResNet50(nn.Module):
    def __init__(self, num_classes: int = 1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        layers, cin = [], 64
        for planes, n, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            blocks = []
            for i in range(n):
                blocks.append(_Bottleneck(cin, planes, stride if i == 0 else 1, i == 0))
                cin = planes * 4
            layers.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = layers
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


# ---------------------------------------------------------------- BERT-base (HF-equivalent)
class _BertLayer(nn.Module):
    def __init__(self, h: int, heads: int, inter: int, p: float):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(h, 3 * h)
        self.out = nn.Linear(h, h)
        self.ln1 = nn.LayerNorm(h, eps=1e-12)
        self.ffn1 = nn.Linear(h, inter)
        self.ffn2 = nn.Linear(inter, h)
        self.ln2 = nn.LayerNorm(h, eps=1e-12)
        self.act = nn.GELU()
        self.drop = nn.Dropout(p)
        self.p = p

    def forward(self, x, mask):
        B, S, H = x.shape
        q, k, v = self.qkv(x).view(B, S, 3, self.heads, H // self.heads).permute(2, 0, 3, 1, 4)
        ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=self.p if self.training else 0.0)
        ctx = ctx.transpose(1, 2).reshape(B, S, H)
        x = self.ln1(x + self.drop(self.out(ctx)))
        return self.ln2(x + self.drop(self.ffn2(self.act(self.ffn1(x)))))


class StockBert(nn.Module):
    def __init__(self, vocab: int = 30522, h: int = 768, layers: int = 12, heads: int = 12, inter: int = 3072,
                 max_pos: int = 512, num_labels: int = 2, p: float = 0.1):
        super().__init__()
        self.word = nn.Embedding(vocab, h)
        self.pos = nn.Embedding(max_pos, h)
        self.typ = nn.Embedding(2, h)
        self.ln = nn.LayerNorm(h, eps=1e-12)
        self.drop = nn.Dropout(p)
        self.layers = nn.ModuleList([_BertLayer(h, heads, inter, p) for _ in range(layers)])
        self.pooler = nn.Linear(h, h)
        self.cls = nn.Linear(h, num_labels)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)
                if isinstance(m, nn.Linear):
                    nn.init.zeros_(m.bias)

    def forward(self, ids, attention_mask=None):
        B, S = ids.shape
        x = self.word(ids) + self.pos.weight[:S].unsqueeze(0) + self.typ.weight[0]
        x = self.drop(self.ln(x))
        mask = None
        if attention_mask is not None:
            mask = ((1.0 - attention_mask[:, None, None, :].to(x.dtype)) * -10000.0)
        for layer in self.layers:
            x = layer(x, mask)
        pooled = torch.tanh(self.pooler(x[:, 0]))
        return self.cls(self.drop(pooled))


# ---------------------------------------------------------------- ViT-B/16 (HF-equivalent)
class _ViTLayer(nn.Module):
    def __init__(self, h: int, heads: int, inter: int):
        super().__init__()
        self.heads = heads
        self.ln1 = nn.LayerNorm(h, eps=1e-12)
        self.qkv = nn.Linear(h, 3 * h)
        self.out = nn.Linear(h, h)
        self.ln2 = nn.LayerNorm(h, eps=1e-12)
        self.ffn1 = nn.Linear(h, inter)
        self.ffn2 = nn.Linear(inter, h)
        self.act = nn.GELU()

    def forward(self, x):
        B, S, H = x.shape
        q, k, v = self.qkv(self.ln1(x)).view(B, S, 3, self.heads, H // self.heads).permute(2, 0, 3, 1, 4)
        ctx = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, S, H)
        x = x + self.out(ctx)
        return x + self.ffn2(self.act(self.ffn1(self.ln2(x))))


class StockViT(nn.Module):
    def __init__(self, image: int = 224, patch: int = 16, h: int = 768, layers: int = 12, heads: int = 12,
                 inter: int = 3072, num_classes: int = 1000):
        super().__init__()
        n = (image // patch) ** 2
        self.patch = nn.Conv2d(3, h, patch, patch)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, h))
        self.pos = nn.Parameter(torch.randn(1, n + 1, h) * 0.02)
        self.layers = nn.ModuleList([_ViTLayer(h, heads, inter) for _ in range(layers)])
        self.ln = nn.LayerNorm(h, eps=1e-12)
        self.head = nn.Linear(h, num_classes)

    def forward(self, x):
        t = self.patch(x).flatten(2).transpose(1, 2)
        t = torch.cat([self.cls_token.expand(x.shape[0], -1, -1).to(t.dtype), t], 1) + self.pos.to(t.dtype)
        for layer in self.layers:
            t = layer(t)
        return self.head(self.ln(t)[:, 0])


# ---------------------------------------------------------------- LAMB on torch._foreach ops
class ForeachLAMB(torch.optim.Optimizer):
    """LAMB (You et al.) as a stock PyTorch user writes it: multi-tensor ``_foreach`` ops,
    per-tensor trust ratio ||p|| / ||update||, global-norm clipping of the gradient first."""

    def __init__(self, params, lr=2e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_grad_norm=1.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.max_grad_norm = max_grad_norm

    @torch.no_grad()
    def step(self, closure=None):
        for grp in self.param_groups:
            ps = [p for p in grp["params"] if p.grad is not None]
            if not ps:
                continue
            gs = [p.grad.float() for p in ps]
            if self.max_grad_norm:
                norm = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(gs)))
                torch._foreach_mul_(gs, torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0))
            for p in ps:
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["m"] = torch.zeros_like(p, dtype=torch.float32)
                    st["v"] = torch.zeros_like(p, dtype=torch.float32)
            ms = [self.state[p]["m"] for p in ps]
            vs = [self.state[p]["v"] for p in ps]
            b1, b2 = grp["betas"]
            t = self.state[ps[0]]["step"] + 1
            for p in ps:
                self.state[p]["step"] = t
            torch._foreach_mul_(ms, b1)
            torch._foreach_add_(ms, gs, alpha=1 - b1)
            torch._foreach_mul_(vs, b2)
            torch._foreach_addcmul_(vs, gs, gs, value=1 - b2)
            mh = torch._foreach_div(ms, 1 - b1 ** t)
            vh = torch._foreach_div(vs, 1 - b2 ** t)
            torch._foreach_sqrt_(vh)
            torch._foreach_add_(vh, grp["eps"])
            upd = torch._foreach_div(mh, vh)
            p32 = [p.float() for p in ps]
            if grp["weight_decay"]:
                torch._foreach_add_(upd, p32, alpha=grp["weight_decay"])
            pn = torch._foreach_norm(p32)
            un = torch._foreach_norm(upd)
            ratios = [torch.where((a > 0) & (b > 0), a / b, torch.ones_like(a)) for a, b in zip(pn, un)]
            torch._foreach_mul_(upd, ratios)
            torch._foreach_add_(p32, upd, alpha=-grp["lr"])
            for p, q in zip(ps, p32):
                if q.data_ptr() != p.data_ptr():
                    p.copy_(q)


# ---------------------------------------------------------------- runner
def run_stock(model: str, batch: int, steps: int, warmup: int, seq_len: int = 128, dropout: float = 0.1,
              seed: int = 1234, bucket_mb: float = 25.0, pad_fraction: float = 0.0,
              grad_accum: int = 1) -> Dict[str, Any]:
    """Train ``model`` ("resnet50" | "bert_base" | "vit_b16" | "bert_large") with stock PyTorch +
    torch DDP on this rank's device; returns the same summary fields as
    ``training.loop.Trainer.run``.  ``grad_accum`` micro-batches per optimizer step (DDP
    ``no_sync`` on all but the last)."""
    from ..parallel import dist as ddist
    dev = ddist.device()
    rank, world = ddist.rank(), ddist.world_size()
    torch.manual_seed(seed)
    g = torch.Generator(device=dev)
    g.manual_seed(seed * 1000 + rank)
    cuda = dev.type == "cuda"
    if model == "resnet50":
        net = StockResNet50().to(dev).to(memory_format=torch.channels_last)
        data = [(torch.randn(batch, 3, 224, 224, generator=g, device=dev).to(memory_format=torch.channels_last),
                 torch.randint(0, 1000, (batch,), generator=g, device=dev)) for _ in range(4)]
        opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5,
                              **({"fused": True} if cuda else {}))

        def loss_fn(m, b):
            return F.cross_entropy(m(b[0]), b[1])
        optimizer = "sgd"
    elif model == "vit_b16":
        net = StockViT().to(dev).to(memory_format=torch.channels_last)
        data = [(torch.randn(batch, 3, 224, 224, generator=g, device=dev).to(memory_format=torch.channels_last),
                 torch.randint(0, 1000, (batch,), generator=g, device=dev)) for _ in range(4)]
        opt = torch.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.05, **({"fused": True} if cuda else {}))

        def loss_fn(m, b):
            return F.cross_entropy(m(b[0]), b[1])
        optimizer = "adamw"
    elif model in ("bert_base", "bert_large"):
        large = model == "bert_large"
        net = (StockBert(h=1024, layers=24, heads=16, inter=4096, p=dropout) if large else StockBert(p=dropout)).to(dev)

        def mask():
            if pad_fraction <= 0:
                return None
            lens = torch.randint(int(seq_len * (1 - pad_fraction)), seq_len + 1, (batch,), generator=g, device=dev)
            return (torch.arange(seq_len, device=dev)[None, :] < lens[:, None]).to(torch.int64)
        data = [(torch.randint(0, 30522, (batch, seq_len), generator=g, device=dev),
                 torch.randint(0, 2, (batch,), generator=g, device=dev), mask()) for _ in range(4)]
        if large:
            opt = ForeachLAMB(net.parameters(), lr=2e-3, weight_decay=0.01)
        else:
            opt = torch.optim.AdamW(net.parameters(), lr=2e-5, weight_decay=0.01, eps=1e-6,
                                    **({"fused": True} if cuda else {}))

        def loss_fn(m, b):
            return F.cross_entropy(m(b[0], b[2]), b[1])
        optimizer = "lamb" if large else "adamw"
    else:
        raise KeyError(model)
    n_params = sum(p.numel() for p in net.parameters())
    ddp = nn.parallel.DistributedDataParallel(net, device_ids=[dev.index] if cuda else None,
                                              bucket_cap_mb=bucket_mb, gradient_as_bucket_view=True)
    amp = torch.autocast(device_type="cuda" if cuda else "cpu", dtype=torch.bfloat16)

    def step(i):
        opt.zero_grad(set_to_none=True)
        for a in range(grad_accum):
            ctx = ddp.no_sync() if a < grad_accum - 1 else contextlib.nullcontext()
            with ctx:
                with amp:
                    loss = loss_fn(ddp, data[(i * grad_accum + a) % len(data)])
                loss.backward()
        opt.step()
        return loss

    ddp.train()
    for i in range(warmup):
        step(i)

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)
    ddist.barrier()
    sync()
    t0 = time.perf_counter()
    loss = None
    for i in range(steps):
        loss = step(warmup + i)
    ddist.barrier()
    sync()
    t = time.perf_counter() - t0
    t_max = ddist.all_reduce_scalars([t], op="max")[0]
    lv = float(loss) if loss is not None else math.nan
    out = {
        "model": model, "task": "cv" if model in ("resnet50", "vit_b16") else "nlp", "world_size": world,
        "steps": steps, "warmup": warmup, "per_rank_batch": batch, "grad_accum": grad_accum,
        "global_batch": batch * world * grad_accum,
        "seq_len": seq_len if model not in ("resnet50", "vit_b16") else None, "dtype": "bf16", "optimizer": optimizer,
        "params": n_params, "seconds": t_max, "ms_per_step": 1000.0 * t_max / max(1, steps),
        "samples_per_sec": batch * world * grad_accum * steps / t_max if t_max > 0 else 0.0, "final_loss": lv,
        "native": "stock", "comm": "torch-ddp",
    }
    if cuda:
        out["mem_peak_gb"] = torch.cuda.max_memory_allocated(dev) / 2**30
    return out
