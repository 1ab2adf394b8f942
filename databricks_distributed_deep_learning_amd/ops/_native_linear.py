"""Linear layer on the MFMA GEMM (csrc/kernels/gemm.hip), with autograd.

forward : y = act(x W^T + b)      mode NT, bias+act in the epilogue; with GELU the
          pre-activation z is written by the same epilogue for backward
backward: dz = dy * act'(z)       (GELU: ddl_gelu_bwd; tanh/relu from the output)
          dx = dz W               mode NN (W read reduction-outer through the
                                  LDS transpose reads; no W^T copy)
          dW = dz^T x             mode TN, split-K over tokens
          db = colsum(dz)
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _lib
from ._lib import call, dcode, grad_ready, grad_sink, p
from ._native_gemm import MODE_NN, MODE_NT, MODE_TN, gemm, stats_rows_max
from . import _native_elementwise as E


def _ok(x, w) -> bool:
    K = x.shape[-1]
    N = w.shape[0]
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and K % 8 == 0 and N % 8 == 0
            and x.numel() > 0)


def _ok_padded(x, w) -> bool:
    """Output width not a multiple of 8 (a classifier head: num_labels = 2): the GEMMs run on the
    native kernels over N rounded up to 8 (zero weight rows), see ``_LinearPadN``."""
    K = x.shape[-1]
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and K % 8 == 0 and w.shape[0] % 8 != 0
            and x.numel() > 0)


class _LinearPadN(torch.autograd.Function):
    """y = x W^T (+ b) (tanh / relu) for N % 8 != 0 on the native GEMMs: W, b and dy are
    zero-padded to Np = roundup(N, 8) rows / columns (a few KB for a classifier head), so the
    forward NT, the dgrad NN (reduction over Np) and the weight-gradient TN are the same
    MFMA kernels as every other Linear -- no vendor GEMM runs for the head.  The padded W / b are
    cached per parameter version (rebuilt once per optimizer step), every pad / slice is one native
    ``ddl_copy2d`` launch, and the gradients go straight into the arena slots."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        K, N = x.shape[-1], w.shape[0]
        Np = (N + 7) // 8 * 8
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M = x2.shape[0]
        wp, bp = _padded(w, b, Np)
        y = torch.empty(M, Np, dtype=x.dtype, device=x.device)
        gemm(MODE_NT, x2, K, wp, K, y, Np, M, Np, K, bias=bp, act=act if act in ("tanh", "relu") else None)
        out = E.copy2d(torch.empty(M, N, dtype=x.dtype, device=x.device), y, N, M, N, Np, M, N)
        ctx.save_for_backward(x2, wp, out if act in ("tanh", "relu") else None)
        ctx.act, ctx.has_bias, ctx.xshape, ctx.N = act, b is not None, x.shape, N
        ctx.w_param, ctx.b_param = w, b
        return out.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, wp, y = ctx.saved_tensors
        M, K = x2.shape
        N, Np = ctx.N, wp.shape[0]
        dy2 = dy.reshape(M, N)
        if ctx.act == "tanh":
            dy2 = E.tanh_bwd(dy2, y)
        elif ctx.act == "relu":
            dy2 = dy2 * (y > 0)
        dy2 = dy2.contiguous()
        dyp = E.copy2d(torch.empty(M, Np, dtype=dy2.dtype, device=dy2.device), dy2, Np, M, Np, N, M, N)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=x2.dtype, device=x2.device)
            gemm(MODE_NN, dyp, Np, wp, K, dx, K, M, K, Np)
            dx = dx.view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dwp = torch.empty(Np, K, dtype=wp.dtype, device=wp.device)
            gemm(MODE_TN, dyp, Np, x2, K, dwp, K, Np, K, M)
            sink = grad_sink(ctx.w_param)
            if sink is not None and sink.dtype == dwp.dtype:
                E.add_into(sink.view(-1), dwp[:N].reshape(-1))     # rows 0..N-1: contiguous
                grad_ready(ctx.w_param)
            else:
                dw = dwp[:N]
        if ctx.has_bias and ctx.needs_input_grad[2]:
            dbp = torch.empty(Np, dtype=wp.dtype, device=wp.device)
            E.colsum(dyp, dbp)
            sink = grad_sink(ctx.b_param)
            if sink is not None and sink.dtype == dbp.dtype:
                E.add_into(sink.view(-1), dbp[:N])
                grad_ready(ctx.b_param)
            else:
                db = dbp[:N]
        return dx, dw, db, None


def _padded(w: torch.Tensor, b: Optional[torch.Tensor], Np: int):
    """W zero-padded to Np rows (and b to Np), cached on the parameter until its values change (the
    same version key as the W^T cache below)."""
    ref = getattr(w, "_ddl_arena", None)
    arena = ref() if ref is not None else None
    key = (w.data_ptr(), w._version, Np, arena.generation if arena is not None else -1,
           None if b is None else (b.data_ptr(), b._version))
    c = getattr(w, "_ddl_padn", None)
    if c is not None and c[0] == key:
        return c[1], c[2]
    N, K = w.shape
    wc = w.contiguous()
    wp = E.copy2d(torch.empty(Np, K, dtype=w.dtype, device=w.device), wc, K, Np, K, K, N, K)
    bp = None
    if b is not None:
        bp = E.copy2d(torch.empty(Np, dtype=b.dtype, device=b.device), b.contiguous(), Np, 1, Np, N, 1, N)
    try:
        w._ddl_padn = (key, wp, bp)
    except (AttributeError, RuntimeError):
        pass
    return wp, bp


# dgrad as an NT GEMM against a cached W^T (DDL_DGRAD_NT=1) or as NN with W read through
# transposed LDS reads (default): since the NN kernel's ds_read_b64_tr_b16 no longer waits
# out the operand prefetch, NN is as fast as NT and needs no per-step W^T copy (the copy
# is rebuilt after every optimizer step: 51 transposes, 0.6 ms per BERT-base step)
_DGRAD_NT = os.environ.get("DDL_DGRAD_NT", "0") != "0"


def _transposed(param, w: torch.Tensor) -> torch.Tensor:
    """W^T for the NT dgrad, cached on the parameter until the weights change: one
    transpose per optimizer step instead of one per backward.  An in-place torch update
    bumps ``w._version``; the flat optimizers write the arena behind the views' version
    counters and bump the arena's ``generation`` instead, so the key holds both."""
    ref = getattr(param, "_ddl_arena", None) if param is not None else None
    arena = ref() if ref is not None else None
    key = (w.data_ptr(), w._version, tuple(w.shape), arena.generation if arena is not None else -1)
    c = getattr(param, "_ddl_wt", None) if param is not None else None
    if c is not None and c[0] == key:
        return c[1]
    wt = w.t().contiguous()
    if param is not None:
        param._ddl_wt = (key, wt)
    return wt


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, bridge=None, fuse_dgelu=False, residual=None, res_bridge=None):
        ctx.w_param, ctx.b_param = w, b
        ctx.bridge = bridge
        ctx.res_bridge = res_bridge if residual is not None else None
        # GELU chain (FFN): this layer's input is the output of a GELU Linear whose only
        # consumer is this layer -> the dgrad epilogue applies that layer's dGELU and
        # column-sums the result (its bias gradient); see ``_DgeluHandoff``
        pre = getattr(x, "_ddl_gelu_pre", None) if fuse_dgelu else None
        ctx.gelu_pre = pre
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        w = w.contiguous()
        M = x2.shape[0]
        y = torch.empty(M, N, dtype=x.dtype, device=x.device)
        z = None
        if act == "gelu" and any(ctx.needs_input_grad[:3]):   # grad mode is off inside forward
            z = torch.empty_like(y)
        res = None
        if residual is not None:
            res = residual.reshape(M, N)
            if not res.is_contiguous() or res.dtype != y.dtype:
                res = res.contiguous().to(y.dtype)
        gemm(MODE_NT, x2, K, w, K, y, N, M, N, K, bias=b, act=act, aux=z, residual=res)
        ctx.act = act
        ctx.has_res = residual is not None
        ctx.has_bias = b is not None
        ctx.save_for_backward(x2, w, z if act == "gelu" else (y if act in ("tanh", "relu") else None))
        ctx.xshape = x.shape
        out = y.view(*x.shape[:-1], N)
        if z is not None:
            ctx.gelu_token = object()
            out._ddl_gelu_pre = (z, ctx.gelu_token)
        elif b is not None and act is None:
            # a LayerNorm consuming ``out`` may add the column sums of its input gradient
            # (this bias's gradient) straight into the bias's arena slot (with a residual too:
            # the residual does not change the bias gradient; if autograd sums another branch
            # into ``out``'s gradient, the backward below corrects the sunk share)
            out._ddl_bias_param = b
        return out

    @staticmethod
    def backward(ctx, dy):
        x2, w, saved = ctx.saved_tensors
        M, K = x2.shape
        N = w.shape[0]
        # the residual's gradient is dy itself (identity add in the epilogue); handed to the
        # LayerNorm that also consumes the residual when a bridge joins them
        dres = dy if ctx.has_res else None
        if dres is not None and ctx.res_bridge is not None:
            ctx.res_bridge.put(dres)
            dres = None
        ctx.res_bridge = None
        dy2 = dy.reshape(M, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        bias_done = False
        handoff = getattr(dy, "_ddl_dgelu_done", None) if ctx.act == "gelu" else None
        if handoff is not None and (handoff.token is not getattr(ctx, "gelu_token", None)
                                    or handoff.version != dy._version):
            handoff = None
        if handoff is not None:
            # the consumer's dgrad already produced dZ = dH * GELU'(z) and its column sums
            dz = dy2
            if ctx.has_bias and ctx.needs_input_grad[2]:
                db_ret = handoff.bias_grad(ctx.b_param, N)
                bias_done = True
        elif ctx.act == "gelu":
            dz = torch.empty_like(dy2)
            if ctx.has_bias and ctx.needs_input_grad[2]:
                # dGELU and the bias gradient (column sums of dz) in one pass
                sink = grad_sink(ctx.b_param)
                db_out = sink if sink is not None else torch.empty(N, dtype=w.dtype, device=w.device)
                nblk = _lib.fn("ddl_colsum_nblk")(M)
                part = torch.empty(nblk * N, dtype=torch.float32, device=dy2.device)
                call("ddl_gelu_bwd_colsum", dcode(dy2), p(dy2), p(saved), p(dz), M, N, p(part), p(db_out),
                     dcode(db_out), int(sink is not None))
                if sink is not None:
                    grad_ready(ctx.b_param)
                    db_ret = None
                else:
                    db_ret = db_out
                bias_done = True
            else:
                call("ddl_gelu_bwd", dcode(dy2), p(dy2), p(saved), p(dz), dz.numel())
        elif ctx.act == "tanh":
            dz = E.tanh_bwd(dy2, saved)
        elif ctx.act == "relu":
            dz = dy2 * (saved > 0)
        else:
            dz = dy2
        # DDL_WGRAD_STREAM: the wgrad below starts from HERE on the side stream, concurrent
        # with the dgrad (whose grid leaves CUs idle at N = 768: 192 tiles on 256 CUs)
        fork = _lib.fork_event() if ctx.needs_input_grad[1] else None
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=x2.dtype, device=x2.device)
            # a residual branch's gradient handed over by the LayerNorm backward: summed
            # in the dgrad epilogue (one extra read instead of an autograd add kernel)
            res = ctx.bridge.take() if ctx.bridge is not None else None
            if res is not None:
                res = res.reshape(M, K)
                if not res.is_contiguous() or res.dtype != dx.dtype:
                    res = res.contiguous().to(dx.dtype)
            pre = ctx.gelu_pre
            fused = None
            if pre is not None and res is None and pre[0].shape == (M, K) and _dgelu_fusable(K):
                # dx := dZ of the producing GELU Linear (dGELU + its bias column sums in the epilogue)
                part = torch.empty(stats_rows_max(M) * 2 * K, dtype=torch.float32, device=dx.device)
                # (tuned among the kernels with a register dGELU epilogue: big, big192, duo)
                if _DGRAD_NT and M >= 4 * K:
                    nrows = gemm(MODE_NT, dz, N, _transposed(ctx.w_param, w), N, dx, K, M, K, N, act="dgelu",
                                 aux=pre[0], colstats=part)
                else:
                    nrows = gemm(MODE_NN, dz, N, w, K, dx, K, M, K, N, act="dgelu", aux=pre[0], colstats=part)
                fused = _DgeluHandoff(pre[1], part, nrows, K)
            elif _DGRAD_NT and M >= 4 * K:
                # dx = dz W as an NT GEMM against W^T (both operands k-contiguous: ds_read_b128
                # fragments instead of transposed reads); the weight copy is tiny next to dz
                gemm(MODE_NT, dz, N, _transposed(ctx.w_param, w), N, dx, K, M, K, N, residual=res)
            else:
                gemm(MODE_NN, dz, N, w, K, dx, K, M, K, N, residual=res)
            dx = dx.view(ctx.xshape)
            if fused is not None:
                fused.version = dx._version
                dx._ddl_dgelu_done = fused
        elif ctx.bridge is not None:
            ctx.bridge.take()
        if ctx.needs_input_grad[1]:
            sink = grad_sink(ctx.w_param)
            if sink is None:
                dw = torch.empty(N, K, dtype=w.dtype, device=w.device)
            # concurrent with the dgrad just issued (DDL_WGRAD_STREAM, _lib.side_stream)
            with _lib.side_stream(dz, x2, after=fork):
                if sink is not None:       # accumulate straight into the reducer's gradient arena
                    gemm(MODE_TN, dz, N, x2, K, sink, K, N, K, M, accumulate=True)
                else:
                    gemm(MODE_TN, dz, N, x2, K, dw, K, N, K, M)
            if sink is not None:
                grad_ready(ctx.w_param)
        sunk = getattr(ctx.b_param, "_ddl_sunk", None) if ctx.has_bias else None
        if sunk is not None:
            ctx.b_param._ddl_sunk = None
        if bias_done:
            db = db_ret
        elif sunk is not None and ctx.needs_input_grad[2]:
            # a LayerNorm backward already added its input gradient's column sums to the bias
            # gradient; if dy is not exactly that gradient (autograd summed another branch in),
            # add the full column sums and take the LayerNorm's share back out
            pre = getattr(dy, "_ddl_colsum", None)
            if ctx.act is not None or pre is None or pre[0] is not sunk or pre[1] != dy._version:
                sink = grad_sink(ctx.b_param)
                E.colsum(dz, sink, accumulate=True)
                sink.copy_(sink.float() - sunk)
            grad_ready(ctx.b_param)
        elif ctx.has_bias and ctx.needs_input_grad[2]:
            sink = grad_sink(ctx.b_param)
            # a LayerNorm backward that produced dy already summed its columns
            pre = getattr(dy, "_ddl_colsum", None) if ctx.act is None else None
            pre = pre[0] if (pre is not None and pre[1] == dy._version) else None
            if pre is not None and pre.numel() == N:
                if sink is not None:
                    call("ddl_acc_f32", dcode(sink), p(sink), p(pre), N)
                    grad_ready(ctx.b_param)
                else:
                    db = pre.to(w.dtype)
            elif (rows := _colsum_rows(dy, ctx.act, N)) is not None:
                # per-batch column sums from the attention backward that produced dy
                out = sink if sink is not None else torch.empty(N, dtype=w.dtype, device=w.device)
                ws = torch.empty(-(-rows.shape[0] // 32) * N, dtype=torch.float32, device=rows.device)
                call("ddl_rows_sum_sink", dcode(out), p(rows), rows.shape[0], N, N, p(out), int(sink is not None),
                     p(ws))
                if sink is not None:
                    grad_ready(ctx.b_param)
                else:
                    db = out
            elif sink is not None:
                E.colsum(dz, sink, accumulate=True)
                grad_ready(ctx.b_param)
            else:
                db = torch.empty(N, dtype=w.dtype, device=w.device)
                E.colsum(dz, db)
        return dx, dw, db, None, None, None, dres, None


def _colsum_rows(dy, act, N):
    """The [rows, N] fp32 column-sum rows riding on ``dy`` (attention backward), if they
    describe exactly this gradient (no activation in between, untouched since)."""
    r = getattr(dy, "_ddl_colsum_rows", None)
    if r is None or act is not None or r[1] != dy._version or r[0].dim() != 2 or r[0].shape[1] != N:
        return None
    return r[0]


def _dgelu_fusable(K: int) -> bool:
    """dGELU + column sums exist on the 256x256 kernel's register epilogue only."""
    from . import _native_gemm as NG
    return os.environ.get("DDL_GEMM_DIRECT", "1") != "0" and NG._big_allowed(MODE_NT, K) and K % 4 == 0


class _DgeluHandoff:
    """Rides on the gradient a GELU-chain consumer returns: the gradient is already
    dZ = dH * GELU'(z) of the producing Linear, whose bias gradient is the column sum
    held in ``part`` (one [sum | sumsq] row per 128 output rows).  ``token`` ties it to
    that producer's forward, ``version`` guards against autograd accumulating anything
    else into the tensor."""
    __slots__ = ("token", "part", "nrows", "width", "version")

    def __init__(self, token, part, nrows, width):
        self.token, self.part, self.nrows, self.width, self.version = token, part, nrows, width, -1

    def bias_grad(self, b_param, N: int):
        ws = torch.empty(-(-self.nrows // 32) * 2 * self.width, dtype=torch.float32, device=self.part.device)
        sink = grad_sink(b_param)
        if sink is not None:
            # column sums accumulated straight into the bias's gradient slot
            call("ddl_rows_sum_sink", dcode(sink), p(self.part), self.nrows, 2 * self.width, N, p(sink), 1, p(ws))
            grad_ready(b_param)
            return None
        row = torch.empty(2 * self.width, dtype=torch.float32, device=self.part.device)
        call("ddl_bn_rows_sum", p(self.part), self.nrows, 2 * self.width, p(row), p(ws))
        return row[:N].to(b_param.dtype)


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], act: Optional[str],
           bridge=None, fuse_dgelu: bool = False, residual: Optional[torch.Tensor] = None,
           residual_grad_to=None) -> torch.Tensor:
    if (_ok_padded(x, w) and bridge is None and residual is None and act in (None, "tanh", "relu")
            and (b is None or b.dtype == w.dtype)):
        return _LinearPadN.apply(x, w, b, act)
    if not _ok(x, w) or (b is not None and b.dtype != w.dtype) or \
            (residual is not None and residual.shape[-1] != w.shape[0]):
        from .bridge import join
        from .linear import linear_reference
        y = linear_reference(join(x, bridge), w, b, act)
        return y if residual is None else y + residual
    return _Linear.apply(x, w, b, act, bridge, fuse_dgelu, residual, residual_grad_to)
