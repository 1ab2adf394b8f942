"""Autograd bindings for the HIP BatchNorm / LayerNorm kernels (csrc/kernels/norm.hip)."""
from __future__ import annotations

import os
from types import SimpleNamespace
from typing import Optional

import torch

from . import _lib
from ._native_elementwise import new_seed
from ._lib import call, dcode, grad_ready, grad_sink, p

# BatchNorm backward reduction in the dgrad epilogue of the conv that consumes the BN
# output (ops/bridge.py BNBackward); DDL_BN_BWD_EPI=0 keeps the separate partial pass
_BN_BWD_EPI = os.environ.get("DDL_BN_BWD_EPI", "1") != "0"
# ... also when the dgrad adds a bridged residual gradient ("1", default; "nores" skips
# them): on its own the fused epilogue was neutral there (three extra operand streams per
# output site, profiles/bn_bwd_epilogue_ab.log), but its output dz IS the residual gradient
# the BN hands on, so the BN backward no longer writes a copy (+0.3-0.8 % ResNet-50)
_BN_BWD_EPI_RES = os.environ.get("DDL_BN_BWD_EPI", "1") not in ("0", "nores")


# LayerNorm backward adds its input gradient's column sums (the producing Linear's bias
# gradient) straight into that bias's arena slot (DDL_LN_BIAS_SINK=0: the Linear adds them)
_LN_BIAS_SINK = os.environ.get("DDL_LN_BIAS_SINK", "1") != "0"


def _bn_supported(C: int) -> bool:
    return C % 8 == 0 and 256 % (C // 8) == 0


def _group_sum(row: torch.Tensor, group) -> None:
    """In-place SUM all-reduce of a small fp32 row over the SyncBatchNorm group.

    When the data-parallel reducer drives the native RCCL engine over the whole world,
    the row goes through that SAME engine (its communicator and comm stream, then the
    compute stream waits for it): one communicator carries every collective issued
    during backward, in the same program order on every rank."""
    import torch.distributed as dist
    from ..parallel import comm as _comm
    eng = _comm.active()
    if eng is not None and row.is_cuda and (group is None or group is dist.group.WORLD
                                            or dist.get_world_size(group) == eng.world):
        eng.wait_upto(eng.all_reduce(row))
        return
    dist.all_reduce(row, op=dist.ReduceOp.SUM, group=group)


def _bn_train_stats(x, weight, bias, running_mean, running_var, momentum, eps, given, stats) -> None:
    """Training statistics of x into stats = [mean | invstd | scale | shift] (running stats
    updated): from the producing GEMM's epilogue partials (``given``) or a statistics pass."""
    C = x.shape[-1]
    M = x.numel() // C
    dt = dcode(x)
    f32 = dict(dtype=torch.float32, device=x.device)
    if given is not None:                          # partials from the producing GEMM's epilogue
        part, nblk = given
        # thousands of partial rows (one per 128 GEMM rows) are first collapsed 32:1
        ws = torch.empty(-(-nblk // 32) * 2 * C, **f32) if nblk > 32 else None
        call("ddl_bn_fwd_from_partials", dt, p(part), nblk, M, C, p(weight), p(bias), p(running_mean),
             p(running_var), float(momentum), float(eps), p(stats[0]), p(stats[1]), p(stats[2]), p(stats[3]),
             p(ws), 0 if ws is None else ws.numel())
    else:
        nblk = _lib.fn("ddl_bn_stats_nblk")(M, C)
        part = torch.empty(nblk * 2 * C, **f32)
        call("ddl_bn_fwd_train", dt, p(x), M, C, p(weight), p(bias), p(running_mean), p(running_var),
             float(momentum), float(eps), p(part), p(stats[0]), p(stats[1]), p(stats[2]), p(stats[3]))


class _BatchNormTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu, residual, bridge=None,
                pre=None, group=None):
        ctx.bridge = bridge
        ctx.group = group
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        dt = dcode(x)
        f32 = dict(dtype=torch.float32, device=x.device)
        stats = torch.empty(4, C, **f32)           # mean, invstd, scale, shift
        given = pre.take_for(x) if pre is not None else None
        if group is not None:
            # SyncBatchNorm: [sum | sumsq] as one row, summed over the group, finalised with
            # the global row count (equal per-rank batches, as data-parallel training runs)
            import torch.distributed as dist
            world = dist.get_world_size(group)
            if given is not None:
                part, nblk = given
                ws = torch.empty(-(-nblk // 32) * 2 * C, **f32)
            else:
                nblk = _lib.fn("ddl_bn_stats_nblk")(M, C)
                part = torch.empty((nblk + -(-nblk // 32)) * 2 * C, **f32)
                call("ddl_bn_stats_partials", dt, p(x), M, C, p(part))
                ws = None
            row = torch.empty(2 * C, **f32)
            call("ddl_bn_rows_sum", p(part), nblk, 2 * C, p(row), p(ws))
            _group_sum(row, group)
            call("ddl_bn_fwd_from_partials", dt, p(row), 1, M * world, C, p(weight), p(bias), p(running_mean),
                 p(running_var), float(momentum), float(eps), p(stats[0]), p(stats[1]), p(stats[2]), p(stats[3]),
                 None, 0)
            ctx.m_total = M * world
        else:
            _bn_train_stats(x, weight, bias, running_mean, running_var, momentum, eps, given, stats)
        res = residual.contiguous() if residual is not None else None
        y = torch.empty_like(x)
        # ReLU: 1 bit per element for the backward instead of re-reading y
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device) if relu else None
        call("ddl_bn_apply", dt, p(x), p(res), p(stats[2]), p(stats[3]), p(y), x.numel(), C, int(relu), p(mask))
        ctx.relu = bool(relu)
        ctx.has_res = residual is not None
        ctx.params = (weight, bias)
        ctx.save_for_backward(x, mask, weight, stats)
        ctx.bnb = None
        if _BN_BWD_EPI and x.dtype == torch.bfloat16:
            # the conv consuming y may run this BN's backward reduction in its dgrad epilogue
            from .bridge import BNBackward
            ctx.bnb = BNBackward(x, mask, stats[0], stats[1])
            y._ddl_bnb = ctx.bnb
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, stats = ctx.saved_tensors
        dx, dgamma, dbeta, dres = _bn_backward(ctx, dy, x, mask, weight, stats)
        return dx, dgamma, dbeta, None, None, None, None, None, dres, None, None, None


def _bn_backward(ctx, dy, x, mask, weight, stats):
    """Training BatchNorm backward -> (dx, dgamma, dbeta, dres).  ``ctx`` carries bnb (the
    dgrad-epilogue hint), group, has_res, relu, params, bridge and m_total (SyncBN)."""
    dy = dy.contiguous()
    C = x.shape[-1]
    M = x.numel() // C
    nblk = _lib.fn("ddl_bn_bwd_nblk")(M, C)
    f32 = dict(dtype=torch.float32, device=x.device)
    # partial rows + room for their 32:1 collapse (see norm.hip collapse_partials)
    part = torch.empty((nblk + -(-nblk // 32)) * 2 * C, **f32)
    coef = torch.empty(3 * C, **f32)
    dx = torch.empty_like(x)
    sg, sb = grad_sink(ctx.params[0]), grad_sink(ctx.params[1])
    direct = sg is not None and sb is not None
    if direct:
        dgamma, dbeta = sg, sb
    else:
        dgamma = torch.empty_like(weight) if weight is not None else None
        dbeta = torch.empty_like(weight) if weight is not None else None
    given = ctx.bnb.take_for(dy) if ctx.bnb is not None else None
    ctx.bnb = None
    dres = torch.empty_like(x) if ctx.has_res and (given is None or ctx.group is not None) else None
    if given is not None:
        # dy is dz (ReLU mask applied) and [sum dz | sum dz*xhat] came from the dgrad epilogue
        gpart, nrows = given
        if ctx.group is not None:
            row = torch.empty(2 * C, **f32)
            call("ddl_bn_rows_sum", p(gpart), nrows, 2 * C, p(row), None)
            local = row.clone()             # dgamma / dbeta stay this rank's partials
            _group_sum(row, ctx.group)
            call("ddl_bn_bwd_finish", dcode(x), p(dy), None, p(x), p(stats[0]), p(stats[1]), p(weight), M,
                 ctx.m_total, C, 0, p(row), p(local), p(dgamma), p(dbeta), p(coef), p(dx), p(dres), int(direct))
        else:
            ws = gpart[nrows * 2 * C:]
            # the residual gradient IS dz (mask applied, no affine): hand on the dgrad's
            # output itself instead of copying it (one write pass per residual block)
            call("ddl_bn_bwd_from_partials", dcode(x), p(gpart), nrows, p(ws), ws.numel(), p(dy), p(x),
                 p(stats[0]), p(stats[1]), p(weight), M, C, p(dgamma), p(dbeta), p(coef), p(dx), None,
                 int(direct))
            if ctx.has_res:
                dres = dy
    elif ctx.group is not None:
        # SyncBatchNorm: [sum dz | sum dz*xhat] summed over the group before the finalize
        call("ddl_bn_bwd_partials", dcode(x), p(dy), p(mask), p(x), p(stats[0]), p(stats[1]), M, C,
             int(ctx.relu), p(part))
        row = torch.empty(2 * C, **f32)
        call("ddl_bn_rows_sum", p(part), nblk, 2 * C, p(row), None)
        # the group sum feeds the dx coefficients only: dgamma / dbeta are per-rank partials
        # (the data-parallel reducer sums them), as in the CPU reference
        local = row.clone()
        _group_sum(row, ctx.group)
        call("ddl_bn_bwd_finish", dcode(x), p(dy), p(mask), p(x), p(stats[0]), p(stats[1]), p(weight), M,
             ctx.m_total, C, int(ctx.relu), p(row), p(local), p(dgamma), p(dbeta), p(coef), p(dx), p(dres),
             int(direct))
    else:
        call("ddl_bn_bwd", dcode(x), p(dy), p(mask), p(x), p(stats[0]), p(stats[1]), p(weight), M, C,
             int(ctx.relu), p(part), p(dgamma), p(dbeta), p(coef), p(dx), p(dres), int(direct))
    if direct:
        grad_ready(ctx.params[0])
        grad_ready(ctx.params[1])
        dgamma = dbeta = None
    if dres is not None and ctx.bridge is not None:
        ctx.bridge.put(dres)            # summed into the consumer's dgrad epilogue
        dres = None
    return dx, dgamma, dbeta, dres


class _BatchNormAddBNTrain(torch.autograd.Function):
    """relu(BN(x) + BN2(x2)) in training: a ResNet downsample block's output, both BatchNorms
    applied in one pass (``ddl_bn_apply2``) instead of writing BN2's output and re-reading it as
    the residual.  Backward: BN's as with a residual, then BN2's from the residual gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, x2, weight2, bias2, running_mean2,
                running_var2, momentum2, eps2, pre=None, pre2=None):
        x, x2 = x.contiguous(), x2.contiguous()
        C = x.shape[-1]
        f32 = dict(dtype=torch.float32, device=x.device)
        stats = torch.empty(4, C, **f32)
        stats2 = torch.empty(4, C, **f32)
        _bn_train_stats(x, weight, bias, running_mean, running_var, momentum, eps,
                        pre.take_for(x) if pre is not None else None, stats)
        _bn_train_stats(x2, weight2, bias2, running_mean2, running_var2, momentum2, eps2,
                        pre2.take_for(x2) if pre2 is not None else None, stats2)
        y = torch.empty_like(x)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device)
        call("ddl_bn_apply2", dcode(x), p(x), p(x2), p(stats[2]), p(stats[3]), p(stats2[2]), p(stats2[3]), p(y),
             x.numel(), C, 1, p(mask))
        ctx.bridge, ctx.group, ctx.relu, ctx.has_res = None, None, True, True
        ctx.params, ctx.params2 = (weight, bias), (weight2, bias2)
        ctx.save_for_backward(x, mask, weight, stats, x2, weight2, stats2)
        ctx.bnb = None
        if _BN_BWD_EPI and x.dtype == torch.bfloat16:
            from .bridge import BNBackward
            ctx.bnb = BNBackward(x, mask, stats[0], stats[1])
            y._ddl_bnb = ctx.bnb
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, stats, x2, weight2, stats2 = ctx.saved_tensors
        dx, dgamma, dbeta, dres = _bn_backward(ctx, dy, x, mask, weight, stats)
        c2 = SimpleNamespace(bnb=None, group=None, has_res=False, relu=False, params=ctx.params2, bridge=None)
        dx2, dgamma2, dbeta2, _ = _bn_backward(c2, dres, x2, None, weight2, stats2)
        return (dx, dgamma, dbeta, None, None, None, None, dx2, dgamma2, dbeta2, None, None, None, None, None, None)


class _BNReluMaxPoolTrain(torch.autograd.Function):
    """Training maxpool3x3/2(relu(BN(x))) -- the ResNet stem -- in one pass over the conv
    output (``ddl_bn_relu_maxpool``: the full-resolution activation is never written).
    Backward: the max-pool gather, then the BatchNorm backward with the ReLU mask."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, pre=None):
        x = x.contiguous()
        N, H, W, C = x.shape
        P, Q = H // 2, W // 2
        stats = torch.empty(4, C, dtype=torch.float32, device=x.device)
        _bn_train_stats(x, weight, bias, running_mean, running_var, momentum, eps,
                        pre.take_for(x) if pre is not None else None, stats)
        y = torch.empty(N, P, Q, C, dtype=x.dtype, device=x.device)
        idx = torch.empty(N, P, Q, C, dtype=torch.uint8, device=x.device)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device)
        call("ddl_bn_relu_maxpool", dcode(x), p(x), p(stats[2]), p(stats[3]), p(y), p(idx), p(mask), N, H, W, C, P, Q)
        ctx.params = (weight, bias)
        ctx.save_for_backward(x, mask, weight, stats, idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, stats, idx = ctx.saved_tensors
        N, H, W, C = x.shape
        dy = dy.contiguous()
        if not _FUSED_STEM_BWD:
            da = torch.empty_like(x)
            call("ddl_maxpool_bwd", dcode(dy), p(dy), p(idx), p(da), N, H, W, C, H // 2, W // 2, 3, 2, 1)
            c = SimpleNamespace(bnb=None, group=None, has_res=False, relu=True, params=ctx.params, bridge=None)
            dx, dgamma, dbeta, _ = _bn_backward(c, da, x, mask, weight, stats)
            return dx, dgamma, dbeta, None, None, None, None, None
        # the max-pool gather evaluated inside both BatchNorm backward passes (ddl_bn_bwd_pool):
        # the full-resolution activation gradient is never written
        nblk = _lib.fn("ddl_bn_bwd_pool_nblk")()
        f32 = dict(dtype=torch.float32, device=x.device)
        part = torch.empty((nblk + -(-nblk // 32)) * 2 * C, **f32)
        coef = torch.empty(3 * C, **f32)
        dx = torch.empty_like(x)
        sg, sb = grad_sink(ctx.params[0]), grad_sink(ctx.params[1])
        direct = sg is not None and sb is not None
        dgamma, dbeta = (sg, sb) if direct else (torch.empty_like(weight), torch.empty_like(weight))
        call("ddl_bn_bwd_pool", dcode(x), p(dy), p(idx), p(mask), p(x), p(stats[0]), p(stats[1]), p(weight), N, H, W,
             C, H // 2, W // 2, p(part), p(dgamma), p(dbeta), p(coef), p(dx), int(direct))
        if direct:
            grad_ready(ctx.params[0])
            grad_ready(ctx.params[1])
            dgamma = dbeta = None
        return dx, dgamma, dbeta, None, None, None, None, None


def bn_relu_maxpool(x, weight, bias, running_mean, running_var, momentum, eps, pre=None):
    """Training maxpool3x3/2/pad1(relu(BN(x))) in one pass; None when not covered."""
    N, H, W, C = x.shape
    if (not _FUSED_STEM or not _bn_supported(C) or x.dtype not in (torch.bfloat16, torch.float32)
            or H % 2 or W % 2 or weight is None):
        return None
    if weight.dtype != x.dtype:
        weight, bias = weight.to(x.dtype), bias.to(x.dtype)
    return _BNReluMaxPoolTrain.apply(x, weight, bias, running_mean, running_var, momentum, eps, pre)


_FUSED_STEM = os.environ.get("DDL_FUSED_STEM", "1") != "0"
# backward of the fused stem with the max-pool gather inside the BN backward passes: saves the
# activation-gradient write but the gathers slow both passes about as much (same-box A/B neutral
# within noise), so the default keeps max-pool backward + BN backward
_FUSED_STEM_BWD = os.environ.get("DDL_FUSED_STEM_BWD", "0") != "0"
_DUAL_BN = os.environ.get("DDL_DUAL_BN", "1") != "0"


def batch_norm_add_bn(x, weight, bias, running_mean, running_var, momentum, eps, x2, weight2, bias2,
                      running_mean2, running_var2, momentum2, eps2, pre=None, pre2=None):
    """Training relu(BN(x) + BN2(x2)) in one apply pass; None when not covered (the caller
    then runs the two BatchNorms separately; DDL_DUAL_BN=0 always)."""
    C = x.shape[-1]
    if (not _DUAL_BN or not _bn_supported(C) or x.dtype not in (torch.bfloat16, torch.float32) or x2.dtype != x.dtype
            or x2.shape != x.shape or weight is None or weight2 is None):
        return None
    if weight.dtype != x.dtype:
        weight, bias = weight.to(x.dtype), bias.to(x.dtype)
    if weight2.dtype != x.dtype:
        weight2, bias2 = weight2.to(x.dtype), bias2.to(x.dtype)
    return _BatchNormAddBNTrain.apply(x, weight, bias, running_mean, running_var, momentum, eps, x2, weight2, bias2,
                                      running_mean2, running_var2, momentum2, eps2, pre, pre2)


class _BatchNormEval(torch.autograd.Function):
    """Inference BN: per-channel affine from running stats (+res)(ReLU), one pass."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, relu, residual):
        x = x.contiguous()
        C = x.shape[-1]
        coeff = torch.empty(2, C, dtype=torch.float32, device=x.device)
        call("ddl_bn_eval_coeffs", dcode(x), C, p(weight), p(bias), p(running_mean), p(running_var), float(eps),
             p(coeff[0]), p(coeff[1]))
        y = torch.empty_like(x)
        res = residual.contiguous() if residual is not None else None
        call("ddl_bn_apply", dcode(x), p(x), p(res), p(coeff[0]), p(coeff[1]), p(y), x.numel(), C, int(relu), None)
        return y


def batch_norm(x, weight, bias, running_mean, running_var, training, momentum, eps, relu, residual, bridge=None,
               pre=None, group=None):
    from .norm import batch_norm_reference, sync_batch_norm_reference
    C = x.shape[-1]
    if not _bn_supported(C) or x.dtype not in (torch.bfloat16, torch.float32):
        if training and group is not None:
            return sync_batch_norm_reference(x, weight, bias, running_mean, running_var, momentum, eps, relu,
                                             residual, group)
        return batch_norm_reference(x, weight, bias, running_mean, running_var, training, momentum, eps, relu,
                                    residual)
    if weight is not None and weight.dtype != x.dtype:
        weight, bias = weight.to(x.dtype), bias.to(x.dtype)
    if training:
        return _BatchNormTrain.apply(x, weight, bias, running_mean, running_var, momentum, eps, relu, residual,
                                     bridge, pre, group)
    if torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad)):
        # eval-mode BN with gradients (frozen-statistics fine-tuning): reference path
        return batch_norm_reference(x, weight, bias, running_mean, running_var, False, momentum, eps, relu,
                                    residual)
    return _BatchNormEval.apply(x, weight, bias, running_mean, running_var, eps, relu, residual)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, residual, drop_p, bridge=None, grad_from=None):
        # the bias of the Linear that produced x
        ctx.bias_param = getattr(x, "_ddl_bias_param", None) if _LN_BIAS_SINK else None
        ctx.grad_from = grad_from
        x = x.contiguous()
        H = x.shape[-1]
        rows = x.numel() // H
        res = residual.contiguous() if residual is not None else None
        res_rows = res.numel() // H if res is not None else rows
        stats = torch.empty(2, rows, dtype=torch.float32, device=x.device)
        y = torch.empty_like(x)
        seed = new_seed() if drop_p > 0.0 else 0
        call("ddl_ln_fwd", dcode(x), p(x), p(res), res_rows, p(weight), p(bias), p(y), p(stats[0]), p(stats[1]),
             rows, H, float(eps), seed, float(drop_p))
        ctx.seed, ctx.drop_p = seed, float(drop_p)
        ctx.bridge = bridge
        ctx.res_shape = residual.shape if residual is not None else None
        ctx.params = (weight, bias)
        ctx.res_rows = res_rows
        ctx.save_for_backward(x, res, weight, stats)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, res, weight, stats = ctx.saved_tensors
        dy = dy.contiguous()
        H = x.shape[-1]
        rows = x.numel() // H
        nblk = _lib.fn("ddl_ln_bwd_nblk")(rows)
        part = torch.empty((nblk + -(-nblk // 32)) * 3 * H, dtype=torch.float32, device=x.device)
        dxsum = torch.empty(H, dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        sg, sb = grad_sink(ctx.params[0]), grad_sink(ctx.params[1])
        direct = sg is not None and sb is not None
        dg, db = (sg, sb) if direct else (torch.empty_like(weight), torch.empty_like(weight))
        # with fused dropout the residual gets the unmasked gradient, x the masked one
        dres_buf = torch.empty_like(x) if ctx.drop_p > 0.0 else None
        # the producing Linear's bias gradient (column sums of dx) straight into its arena slot
        bsink = grad_sink(ctx.bias_param) if (direct and ctx.bias_param is not None) else None
        if bsink is not None and (bsink.numel() != H or bsink.dtype != dg.dtype
                                  or getattr(ctx.bias_param, "_ddl_sunk", None) is not None):
            bsink = None
        # x's gradient from its other consumer (a pre-LN residual branch, handed over by that
        # Linear's backward): added in the same pass, so dx and its column sums are complete
        add = ctx.grad_from.take() if ctx.grad_from is not None else None
        ctx.grad_from = None
        if add is not None:
            add = add.reshape(x.shape)
            if not add.is_contiguous() or add.dtype != x.dtype:
                add = add.contiguous().to(x.dtype)
            if H // 256 > 4:                 # no fused variant: sum afterwards (sinks off)
                bsink, late = None, add
                add = None
            else:
                late = None
        else:
            late = None
        call("ddl_ln_bwd", dcode(x), p(dy), p(x), p(res), ctx.res_rows, p(weight), p(stats[0]), p(stats[1]), p(dx),
             p(part), p(dg), p(db), rows, H, int(direct), p(dxsum), ctx.seed, ctx.drop_p, p(dres_buf), p(bsink),
             p(add))
        if late is not None:
            dx.add_(late)
            dxsum = None
        if bsink is not None:
            ctx.bias_param._ddl_sunk = dxsum     # the Linear's backward only marks it ready
        ctx.bias_param = None
        # the column sums of dx ride along on the gradient tensor: the Linear whose output
        # fed this LayerNorm takes them as its bias gradient instead of re-reading dx
        # (the version guards against autograd accumulating another gradient into dx in place)
        if dxsum is not None:
            dx._ddl_colsum = (dxsum, dx._version)
        if direct:
            grad_ready(ctx.params[0])
            grad_ready(ctx.params[1])
            dg = db = None
        dres = None
        if ctx.res_shape is not None:
            g = dres_buf if dres_buf is not None else dx
            if ctx.res_rows == rows:
                dres = g.view(ctx.res_shape)
                if ctx.bridge is not None:
                    ctx.bridge.put(dres)       # summed into the consuming Linear's dgrad epilogue
                    dres = None
            else:
                # broadcast residual ([1, S, H] against [B, S, H]): its gradient is the sum over the
                # batch -- one native column-sum launch over [B, S * H] (fp32 partials, bf16 out)
                from . import _native_elementwise as E
                dres = torch.empty(ctx.res_rows * H, dtype=dx.dtype, device=dx.device)
                E.colsum(g.reshape(-1, ctx.res_rows * H), dres)
                dres = dres.view(ctx.res_shape)
        return dx, dg, db, None, dres, None, None, None


def layer_norm(x, weight, bias, eps, residual: Optional[torch.Tensor] = None, dropout: float = 0.0,
               residual_grad_to=None, grad_from=None):
    from .norm import layer_norm_reference
    H = x.shape[-1]
    ok = bool(_lib.fn("ddl_ln_supported")(H)) and x.dtype in (torch.bfloat16, torch.float32)
    if residual is not None:
        ok = ok and residual.dtype == x.dtype and residual.shape[-1] == H and \
            (x.numel() // H) % max(1, residual.numel() // H) == 0
        if ok and residual.numel() != x.numel():
            # only leading-dimension broadcast ([1, S, H] against [B, S, H]) is supported
            ok = residual.dim() == x.dim() and all(r in (1, s) for r, s in zip(residual.shape, x.shape)) and \
                residual.shape[0] == 1 and tuple(residual.shape[1:]) == tuple(x.shape[1:])
    if dropout > 0.0 and (residual is None or residual.numel() != x.numel()):
        ok = False                      # fused dropout: full-size residual only
    if not ok:
        if dropout > 0.0:
            from .activation import dropout as _dropout
            x = _dropout(x, dropout, True)
        from .bridge import join
        return layer_norm_reference(join(x, grad_from), weight, bias, eps, residual)
    if weight.dtype != x.dtype:
        weight, bias = weight.to(x.dtype), bias.to(x.dtype)
    return _LayerNorm.apply(x, weight, bias, eps, residual, float(dropout), residual_grad_to, grad_from)
