"""Stem (7x7 / stride-2 RGB conv) space-to-depth helpers and the index contract of the direct
stem kernels (csrc/kernels/stem_conv.hip), on the CPU.

stem_wgrad_reduce_k writes column ``col`` of a workgroup partial [64][256] (tap (r2, s2) * 16 +
space-to-depth channel (dy * 2 + dx) * 4 + c) to weight element [k][2 r2 + dy][2 s2 + dx][c] and
drops columns past R / S / C; stem_fwd_k reads the weight as [64][256] in the same order.  Both
must agree with ``_s2d_weight`` / ``_s2d_weight_grad``."""
import torch
import torch.nn.functional as F

from databricks_distributed_deep_learning_amd.ops import _native_conv as NC


def _kernel_col_map(R, S, C):
    """(col -> (rr, ss, c) or None) exactly as stem_wgrad_reduce_k computes it."""
    out = {}
    for col in range(256):
        tap, sub, c = col >> 4, (col >> 2) & 3, col & 3
        rr, ss = 2 * (tap >> 2) + (sub >> 1), 2 * (tap & 3) + (sub & 1)
        out[col] = (rr, ss, c) if rr < R and ss < S and c < C else None
    return out


def test_reduce_index_map_inverts_space_to_depth_weight():
    torch.manual_seed(0)
    w = torch.randn(64, 7, 7, 3)
    ws = NC._s2d_weight(w).reshape(64, 256)
    cmap = _kernel_col_map(7, 7, 3)
    for col, tgt in cmap.items():
        if tgt is None:
            assert torch.count_nonzero(ws[:, col]) == 0, col      # padded taps / channels are zero
        else:
            rr, ss, c = tgt
            torch.testing.assert_close(ws[:, col], w[:, rr, ss, c])
    # every original weight element is produced by exactly one column
    hit = sorted(t for t in cmap.values() if t is not None)
    assert hit == sorted((r, s, c) for r in range(7) for s in range(7) for c in range(3))


def test_s2d_weight_grad_matches_kernel_reduce_mapping():
    torch.manual_seed(1)
    dws = torch.randn(64, 4, 4, 16)
    g = NC._s2d_weight_grad(dws, (64, 7, 7, 3))
    flat = dws.reshape(64, 256)
    for col, tgt in _kernel_col_map(7, 7, 3).items():
        if tgt is not None:
            rr, ss, c = tgt
            torch.testing.assert_close(g[:, rr, ss, c], flat[:, col])


def test_space_to_depth_conv_equals_strided_conv():
    """The stride-1 4x4 conv of the space-to-depth input is the 7x7 / stride-2 / pad-3 conv (fp64)."""
    torch.manual_seed(2)
    for H, W in ((32, 32), (29, 35)):
        x = torch.randn(2, H, W, 3, dtype=torch.float64)
        w = torch.randn(64, 7, 7, 3, dtype=torch.float64)
        ref = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), stride=2, padding=3).permute(0, 2, 3, 1)
        xs, ws = NC._s2d_input(x, 3), NC._s2d_weight(w)
        y = F.conv2d(xs.permute(0, 3, 1, 2), ws.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
        P, Q = ref.shape[1], ref.shape[2]
        torch.testing.assert_close(y[:, :P, :Q], ref)


def test_direct_stem_paths_gate_on_device_and_shape():
    xs = torch.zeros(2, 115, 115, 16, dtype=torch.bfloat16)
    dy = torch.zeros(2, 112, 112, 64, dtype=torch.bfloat16)
    ws = torch.zeros(64, 4, 4, 16, dtype=torch.bfloat16)
    # CPU tensors never take the HIP kernels
    assert not NC._stem_fwd_ok(xs, ws)
    assert not NC._stem_wgrad_ok(xs, dy, (64, 4, 4, 16), (64, 7, 7, 3))
