"""Fused flat-arena optimizer launches (csrc/kernels/optim.hip)."""
from __future__ import annotations

import torch

from ._lib import call, dcode, p

_BLOCK = 8192


def _table(opt):
    t = getattr(opt, "_native_table", None)
    if t is None:
        rows = []
        for ti, e in enumerate(opt.arena.entries):
            s = 0
            n8 = (e.numel + 7) // 8 * 8   # pads are zero and inside the arena's aligned slot
            while s < n8:
                ln = min(_BLOCK, n8 - s)
                rows.append((e.offset + s, ln, ti, 1 if e.decay else 0))
                s += ln
        t = torch.tensor(rows, dtype=torch.int32, device=opt.arena.device)
        opt._native_table = t
    return t


def _targets(opt):
    """(master fp32, param-copy or None, pdtype)."""
    if opt.master is not None:
        return opt.master, opt.arena.flat, dcode(opt.arena.flat)
    return opt.arena.flat, None, 0


def _scale_tensor(scale, device):
    if isinstance(scale, torch.Tensor):
        return scale.to(device=device, dtype=torch.float32).reshape(1).contiguous()
    return torch.full((1,), float(scale), dtype=torch.float32, device=device)


def sgd(opt, grad, scale):
    tab = _table(opt)
    master, param, pdt = _targets(opt)
    s = _scale_tensor(scale, grad.device)
    call("ddl_sgd_step", dcode(grad), p(grad), p(master), pdt, p(param), p(opt.buf), p(tab), tab.shape[0], p(s),
         float(opt.lr), float(opt.momentum), float(opt.weight_decay), int(opt.nesterov), int(opt.step_count == 1))


def adamw(opt, grad, scale):
    tab = _table(opt)
    master, param, pdt = _targets(opt)
    s = _scale_tensor(scale, grad.device)
    t = opt.step_count
    call("ddl_adamw_step", dcode(grad), p(grad), p(master), pdt, p(param), p(opt.m), p(opt.v), p(tab), tab.shape[0],
         p(s), float(opt.lr), float(opt.b1), float(opt.b2), float(opt.eps), float(opt.weight_decay),
         float(1 - opt.b1 ** t), float(1 - opt.b2 ** t))


def lamb(opt, grad, scale):
    tab = _table(opt)
    master, param, pdt = _targets(opt)
    s = _scale_tensor(scale, grad.device)
    t = opt.step_count
    norms = torch.zeros(2 * len(opt.arena.entries), dtype=torch.float32, device=grad.device)
    bc1 = (1 - opt.b1 ** t) if opt.bias_correction else 1.0
    bc2 = (1 - opt.b2 ** t) if opt.bias_correction else 1.0
    call("ddl_lamb_step", dcode(grad), p(grad), p(master), pdt, p(param), p(opt.m), p(opt.v), p(tab), tab.shape[0],
         p(s), float(opt.lr), float(opt.b1), float(opt.b2), float(opt.eps), float(opt.weight_decay), float(bc1),
         float(bc2), p(norms))


def global_norm(grad):
    out = torch.zeros(1, dtype=torch.float32, device=grad.device)
    n = grad.numel() // 8 * 8
    call("ddl_sumsq", dcode(grad), p(grad), n, p(out))
    if n != grad.numel():
        out += grad[n:].float().pow(2).sum()
    return out.sqrt().reshape(())
