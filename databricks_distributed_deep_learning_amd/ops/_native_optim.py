"""Fused flat-arena optimizer launches (csrc/kernels/optim.hip)."""
from __future__ import annotations

import bisect

import torch

from ._lib import call, dcode, p

_BLOCK = 8192


def _table(opt):
    """Block table over the optimizer's owned ranges: rows (local start, length | decay << 30,
    tensor index, arena - local offset).  Unsharded the local index IS the arena index;
    sharded (ZeRO-1), every owned chunk starts and ends on a 64-element boundary, so rows
    never straddle another rank's elements."""
    t = getattr(opt, "_native_table", None)
    if t is None:
        rows = []
        for lo, hi, off in opt.ranges:
            delta = lo - off
            for ti, e in enumerate(opt.arena.entries):
                n8 = (e.numel + 7) // 8 * 8   # pads are zero and inside the arena's aligned slot
                a, b = max(e.offset, lo), min(e.offset + n8, hi)
                s = a
                while s < b:
                    ln = min(_BLOCK, b - s)
                    rows.append((s - delta, ln | ((1 if e.decay else 0) << 30), ti, delta))
                    s += ln
        if not rows:
            rows.append((0, 0, 0, 0))
        t = torch.tensor(rows, dtype=torch.int32, device=opt.arena.device)
        opt._native_table = t
        opt._native_starts = [r[0] for r in rows]
    return t


def _rows(opt, rng):
    """(table pointer, row count) for the whole table or the rows of local range [lo, hi)
    (range steps: bucket boundaries are tensor boundaries, so whole rows)."""
    tab = _table(opt)
    if rng is None:
        return tab.data_ptr(), tab.shape[0]
    starts = opt._native_starts
    r0, r1 = bisect.bisect_left(starts, rng[0]), bisect.bisect_left(starts, rng[1])
    return tab.data_ptr() + r0 * tab.stride(0) * tab.element_size(), r1 - r0


def _state(t: torch.Tensor, opt) -> int:
    """State tensors are indexed by the table's local start (no shift)."""
    return t.data_ptr()


def _targets(opt):
    """(master fp32 pointer, param-copy or None, pdtype); the kernels write the param copy at
    local index + the row's arena offset."""
    if opt.master is not None:
        return opt.master.data_ptr(), opt.arena.flat, dcode(opt.arena.flat)
    return opt.arena.flat.data_ptr(), None, 0


def _scale_tensor(scale, device):
    if isinstance(scale, torch.Tensor):
        return scale.to(device=device, dtype=torch.float32).reshape(1).contiguous()
    return torch.full((1,), float(scale), dtype=torch.float32, device=device)


def sgd(opt, grad, scale, rng=None):
    tab, nrow = _rows(opt, rng)
    master, param, pdt = _targets(opt)
    s = _scale_tensor(scale, grad.device)
    call("ddl_sgd_step", dcode(grad), p(grad), master, pdt, p(param), _state(opt.buf, opt), tab, nrow, p(s),
         float(opt.lr), float(opt.momentum), float(opt.weight_decay), int(opt.nesterov), int(opt.step_count == 1))


def adamw(opt, grad, scale, rng=None):
    tab, nrow = _rows(opt, rng)
    master, param, pdt = _targets(opt)
    s = _scale_tensor(scale, grad.device)
    t = opt.step_count
    call("ddl_adamw_step", dcode(grad), p(grad), master, pdt, p(param), _state(opt.m, opt), _state(opt.v, opt),
         tab, nrow,
         p(s), float(opt.lr), float(opt.b1), float(opt.b2), float(opt.eps), float(opt.weight_decay),
         float(1 - opt.b1 ** t), float(1 - opt.b2 ** t))


def lamb(opt, grad, scale, rng=None):
    master, param, pdt = _targets(opt)
    s = _scale_tensor(scale, grad.device)
    t = opt.step_count
    if rng is None:
        norms = torch.zeros(2 * len(opt.arena.entries), dtype=torch.float32, device=grad.device)
    else:   # one zeroed per-tensor norm buffer per range-stepped step (each range fills its own tensors)
        scratch = opt._range_scratch
        norms = scratch.get("norms")
        if norms is None:
            norms = scratch["norms"] = torch.zeros(2 * len(opt.arena.entries), dtype=torch.float32,
                                                   device=grad.device)
    bc1 = (1 - opt.b1 ** t) if opt.bias_correction else 1.0
    bc2 = (1 - opt.b2 ** t) if opt.bias_correction else 1.0
    if opt.shard is None:
        tp, nrow = _rows(opt, rng)
        call("ddl_lamb_step", dcode(grad), p(grad), master, pdt, p(param), p(opt.m), p(opt.v), tp, nrow,
             p(s), float(opt.lr), float(opt.b1), float(opt.b2), float(opt.eps), float(opt.weight_decay), float(bc1),
             float(bc2), p(norms))
        return
    tab = _table(opt)
    # sharded: the per-tensor norms of every rank's pieces are summed between the phases
    from ..optim.flat import _sum_over_ranks
    m, v = _state(opt.m, opt), _state(opt.v, opt)
    call("ddl_lamb_phase1", dcode(grad), p(grad), master, m, v, p(tab), tab.shape[0], p(s), float(opt.b1),
         float(opt.b2), float(opt.eps), float(opt.weight_decay), float(bc1), float(bc2), p(norms))
    _sum_over_ranks(norms)
    call("ddl_lamb_phase2", master, pdt, p(param), m, v, p(tab), tab.shape[0], float(opt.lr), float(opt.eps),
         float(opt.weight_decay), float(bc1), float(bc2), p(norms))


def global_norm(grad):
    out = torch.zeros(1, dtype=torch.float32, device=grad.device)
    n = grad.numel() // 8 * 8
    call("ddl_sumsq", dcode(grad), p(grad), n, p(out))
    if n != grad.numel():
        out += grad[n:].float().pow(2).sum()
    return out.sqrt().reshape(())
