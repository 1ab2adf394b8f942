"""Fused attention vs an fp32 PyTorch reference (GPU only), incl. dropout-mask parity."""
import math

import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu

M32 = 0xFFFFFFFF


def _lowbias32(x):
    """ddl_common.h lowbias32 on int64 tensors holding uint32 values."""
    x = x ^ (x >> 16)
    x = (x * 0x7feb352d) & M32
    x = x ^ (x >> 15)
    x = (x * 0x846ca68b) & M32
    return x ^ (x >> 16)


def hash_u32(seed, idx):
    """torch re-implementation of ddl_common.h hash_u32 (two lowbias32 rounds)."""
    a = _lowbias32((idx & M32) ^ (seed & M32))
    return _lowbias32((a + ((idx >> 32) * 0x9E3779B9 & M32) + (seed >> 32)) & M32)


def attn_keep(seed, idx, p):
    """attention.hip attn_hash / attn_keep_half: one lowbias32 round per pair of score
    indices (idx >> 1), each element thresholded on its 16-bit half."""
    pidx = idx >> 1
    x = (pidx & M32) ^ (seed & M32)
    x = (x + ((pidx >> 32) * 0x9E3779B9 & M32) + (seed >> 32)) & M32
    h = _lowbias32(x)
    half = (h >> ((idx & 1) * 16)) & 0xFFFF
    return half >= min(int(p * 65536.0), 65536)


def ref_attention(qkv, H, mask=None, keep=None, p=0.0):
    B, S, hd3 = qkv.shape
    D = hd3 // (3 * H)
    q, k, v = qkv.float().view(B, S, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
    s = q @ k.transpose(-1, -2) / math.sqrt(D)
    if mask is not None:
        s = s + mask.view(B, 1, 1, S)
    pr = torch.softmax(s, -1)
    if keep is not None:
        pr = pr * keep / (1 - p)
    return (pr @ v).permute(0, 2, 1, 3).reshape(B, S, H * D)


@pytest.mark.parametrize("B,S,H", [(2, 128, 12), (3, 197, 2), (2, 256, 3), (1, 129, 2), (1, 64, 4), (2, 100, 3),
                                   (1, 257, 2), (1, 512, 2)])
@pytest.mark.parametrize("masked", [False, True])
def test_attention_fwd_bwd(B, S, H, masked):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_attention as NA
    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3 * H * 64, device=dev).to(torch.bfloat16).requires_grad_(True)
    mask = None
    if masked:
        lens = torch.randint(S // 2, S + 1, (B,), device=dev)
        mask = ((torch.arange(S, device=dev)[None] >= lens[:, None]).float() * -10000.0)
    out = NA.attention(qkv, H, mask, 0.0)
    q32 = qkv.detach().float().requires_grad_(True)
    ref = ref_attention(q32, H, mask)
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item() + 1e-2, err
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g.to(torch.bfloat16).float())
    gerr = (qkv.grad.float() - q32.grad).abs().max().item()
    assert gerr < 3e-2 * q32.grad.abs().max().item() + 1e-2, gerr


@pytest.mark.parametrize("S", [96, 97, 197, 256, 300, 333])   # odd S: pairs of score indices straddle rows; > 128: medium kernels; > 256: tiled
def test_attention_dropout_mask_parity(S):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.ops import _native_attention as NA
    torch.manual_seed(1)
    B, H, p = 2, 3, 0.25
    qkv = torch.randn(B, S, 3 * H * 64, device=dev).to(torch.bfloat16).requires_grad_(True)
    torch.manual_seed(123)
    out = NA.attention(qkv, H, None, p)
    torch.manual_seed(123)
    seed = NA.new_seed()
    bh = torch.arange(B * H, device=dev).view(B, H, 1, 1)
    qi = torch.arange(S, device=dev).view(1, 1, S, 1)
    ki = torch.arange(S, device=dev).view(1, 1, 1, S)
    idx = (bh * S + qi) * S + ki
    keep = attn_keep(seed, idx, p).float()
    assert abs(keep.mean().item() - (1 - p)) < 0.02
    q32 = qkv.detach().float().requires_grad_(True)
    ref = ref_attention(q32, H, None, keep, p)
    assert (out.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item() + 1e-2
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g.to(torch.bfloat16).float())
    assert (qkv.grad.float() - q32.grad).abs().max().item() < 3e-2 * q32.grad.abs().max().item() + 1e-2


@pytest.mark.parametrize("S,sink", [(128, False), (128, True), (100, True), (197, False), (197, True),
                                    (300, True)])
def test_qkv_bias_gradient_from_attention_column_sums(S, sink):
    """The attention backward writes column sums of dQKV -- per batch (fused kernel, S <= 128)
    or per batch and 64-row tile (dKV / dQ kernels, S = 197 / 300, ragged last tile); the QKV
    Linear takes its bias gradient from them (into the DataParallel slot, or a fresh tensor)
    instead of another pass over dQKV."""
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    torch.manual_seed(2)
    B, H, hid = 3, 4, 256
    mod = torch.nn.Module()
    mod.lin = torch.nn.Linear(hid, 3 * H * 64).to(dev).to(torch.bfloat16)
    if sink:
        from databricks_distributed_deep_learning_amd.parallel import DataParallel
        dp = DataParallel(mod, broadcast_init=False, comm="torch")
    x = torch.randn(B, S, hid, device=dev).bfloat16()
    g = torch.randn(B, S, H * 64, device=dev).bfloat16()
    qkv = ops.linear(x, mod.lin.weight, mod.lin.bias, None)
    ops.attention(qkv, H, None, 0.0).backward(g)
    if sink:
        dp.finish()
    got = mod.lin.bias.grad.float()
    b32 = mod.lin.bias.detach().float().requires_grad_(True)
    ref = ref_attention(x.float() @ mod.lin.weight.detach().float().t() + b32, H)
    ref.backward(g.float())
    err = (got - b32.grad).abs().max().item()
    assert err < 2e-2 * b32.grad.abs().max().item() + 1e-2, err
