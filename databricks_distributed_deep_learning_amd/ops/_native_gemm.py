"""Thin wrapper over ``ddl_gemm`` (csrc/kernels/gemm.hip): modes, split-K policy, workspace."""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
from typing import Optional, Sequence

import torch

from . import _lib
from ._lib import I, L, P

_lib.register({"ddl_gemm": [I, P, L, P, L, P, L, I, I, I, P, I, I, P, I, I, P, L, P, I, P, I, P, P],
               "ddl_gemm_n64": [I, P, L, P, L, P, L, I, I, I, P, I, I, P, I, I, P, L, P, I, P, I, P, P],
               "ddl_gemm_big2": [I, P, L, P, L, P, L, I, I, I, P, I, I, P, I, I, P, L, P, I, P, I, P, P, P],
               "ddl_gemm_wgrad": [P, L, P, L, P, L, I, I, I, I, I, P, L, I, P, P, I, P],
               "ddl_stream_wgrad": [P, L, P, L, P, L, I, I, L, I, P, L, P, I, P],
               "ddl_gemm_duo": [I, P, L, P, L, P, L, I, I, I, P, I, P, P, P, P, P],
               "ddl_gemm_duo_tn": [P, L, P, L, P, L, I, I, I, I, I, P, L, P],
               "ddl_gemm_bnb": [P, P, P]})

MODE_NT, MODE_NN, MODE_TN, MODE_CONV, MODE_CONVW = 0, 1, 2, 3, 4
MODE_CONVW_A = 5      # conv wgrad with the im2col operand on the M side (computes dW^T)
TRANS_OUT = 16        # flag: the kernel stores C^T
N192 = 32             # flag (256x256 kernel): 256 x 192 tiles
ACT = {None: 0, "gelu": 1, "relu": 2, "tanh": 3, "dgelu": 4, "bnb": 5}
BM = BN = 128
BK = 64
NUM_CU = 256
_force_small = False
_zero_pages = {}


def set_big_gemm(enabled: bool) -> None:
    """Route GEMMs to the 256x256 8-phase kernel (True, default) or the 128x128 one."""
    global _force_small
    _force_small = not enabled


_forced: Optional[str] = None
_KINDS = ("big", "big192", "hybrid", "small", "narrow", "tnarrow", "wg", "wg2", "swg", "duo")
# per-call device timing for diagnostics (scripts/debug/gemm_trace.py): list of
# (signature, (kernel, splits), start event, end event) while enabled
_trace: Optional[list] = None


def trace(enabled: bool = True) -> Optional[list]:
    """Start (or stop, returning the records) per-GEMM event timing."""
    global _trace
    out = _trace
    _trace = [] if enabled else None
    return out


@contextlib.contextmanager
def force_kernel(kind: Optional[str]):
    """Route every GEMM inside the block to one kernel kind ("big", "small", ... -- see ``gemm``)."""
    global _forced
    prev, _forced = _forced, kind
    try:
        yield
    finally:
        _forced = prev


def _zero_page(device) -> torch.Tensor:
    z = _zero_pages.get(device)
    if z is None:
        z = torch.zeros(128, dtype=torch.bfloat16, device=device)
        _zero_pages[device] = z
    return z


def use_big(mode: int, M: int, N: int, K: int) -> bool:
    """256x256 tiles pay off when neither output side is narrow (tile waste) and
    there is enough work; reduction-outer (wgrad) shapes use split-K instead."""
    if _force_small or K % 8 or K < 128 or min(M, N) < 192 or mode == MODE_CONVW:
        return False
    tiles = (-(-M // 256)) * (-(-N // 256))
    if mode in (MODE_TN, MODE_CONVW):
        return K >= 1024
    return tiles >= 48


def big_splits(M: int, N: int, K: int) -> int:
    """Split-K count for the 256x256 kernel: as many splits as keep every (tile, split)
    block in ONE round on the CUs (floor, not ceil: a 257th block doubles the time)."""
    tiles = (-(-M // 256)) * (-(-N // 256))
    nk = -(-K // BK)
    if tiles >= 200:
        return 1
    return max(1, min(NUM_CU // tiles, nk // 4))


def pick_splits(M: int, N: int, K: int, force: Optional[int] = None) -> int:
    """Split-K only when the tile grid cannot fill the chip; each split keeps >= 8 K-steps.
    At most 2 blocks per CU fit (LDS), so tiles * splits stays <= 2 * NUM_CU: one more
    block than that runs in a second round and doubles the time."""
    if force is not None:
        return max(1, force)
    tiles = -(-M // BM) * -(-N // BN)
    nk = -(-K // BK)
    if tiles >= NUM_CU or nk < 16:
        return 1
    return max(1, min(2 * NUM_CU // tiles, nk // 8))


_HYBRID = os.environ.get("DDL_GEMM_HYBRID", "1") != "0"   # tuner candidate (A/B: 0 = never)
# tuner candidate "big192" (256 x 192 tiles; DDL_GEMM_192=0 drops it): whole rounds where 256-wide
# tiles leave a partial one (N = 768 / 2304 at M = 16384: 256 / 768 tiles instead of 192 / 576).  With
# the retire depth 2 main loop (gemm_big.hip DDL_DEEP_RETIRE) its half-filled quadrant-1 phases no
# longer cost as much as full ones: 16384x768x768 NT 27.2 vs 34.6 us, 16384x2304x768 72.1 vs 95.1 us
# (profiles/gemm_stamps_dr2.log); forcing: kernel="big192".
_BIG192 = os.environ.get("DDL_GEMM_192", "1") == "1"
_DIRECT = os.environ.get("DDL_GEMM_DIRECT", "1") != "0"    # gemm_big.hip register epilogue (big192 needs it)
def hybrid_rows(M: int, N: int, K: int):
    """Row split of a 256x256-tile GEMM whose tile grid ends in a partial round, or None.

    ViT-B/16's N = 768 GEMMs (M = 25216 tokens) have 99 x 3 = 297 tiles: the persistent grid
    runs 256 of them, then 41 CUs run a second tile each while 215 idle -- two full rounds for
    1.16 rounds of work.  The rows are split instead: rows [0, M1) -- whole rounds of tiles --
    run unsplit, and the remaining rows run split-K over the whole chip (their fp32 partials
    reduced with the epilogue), so the tail takes 1/s of a round plus the reduction.  Returns
    (M1, largest useful split); the tuner times the splits against the plain launch."""
    tn = -(-N // 256)
    tm = -(-M // 256)
    tiles = tm * tn
    if tiles <= NUM_CU or K % BK:
        return None
    tm1 = (tiles // NUM_CU) * NUM_CU // tn
    rem = (tm - tm1) * tn
    smax = min(NUM_CU // max(rem, 1), -(-K // BK) // 4)
    if tm1 <= 0 or rem <= 0 or smax < 2:
        return None
    return tm1 * 256, smax


def _at(t, off: int):
    """A one-element view of ``t`` starting ``off`` elements further (only its pointer is used)."""
    return None if t is None else t.as_strided((1,), (1,), t.storage_offset() + off)


def _launch(kind: str, s: int, mode: int, A, lda, B, ldb, C, ldc, M, N, K, bias, act, aux, conv_arr,
            row_remap, residual, accumulate, colstats=None, bnb=None) -> None:
    if kind not in _KINDS:
        # a cached plan entry from another build (e.g. the removed hipBLASLt candidate)
        kind, s = _heuristic(mode, M, N, K, row_remap, lda, ldb)
    if kind == "hybrid":
        # rows [0, M1): whole rounds of unsplit tiles; rows [M1, M): split-K s over the chip
        M1 = hybrid_rows(M, N, K)[0]
        _launch("big", 1, mode, A, lda, B, ldb, C, ldc, M1, N, K, bias, act, aux, conv_arr, False, residual,
                accumulate)
        _launch("big", s, mode, _at(A, M1 * lda), lda, B, ldb, _at(C, M1 * ldc), ldc, M - M1, N, K, bias, act,
                _at(aux, M1 * ldc), conv_arr, False, _at(residual, M1 * ldc), accumulate)
        return
    if kind.startswith("t"):
        # weight-gradient GEMMs computed transposed (operands swapped, C^T stored): a
        # 64-wide output-channel side lands on the tile's N extent (128x64 tiles)
        kind = kind[1:]
        mode = (MODE_CONVW_A if mode == MODE_CONVW else MODE_TN) | TRANS_OUT
        A, lda, B, ldb, M, N = B, ldb, A, lda, N, M
    bias_bf16 = 1 if (bias is not None and bias.dtype == torch.bfloat16) else 0
    out_f32 = 1 if C.dtype == torch.float32 else 0
    if kind == "swg":
        if (mode == MODE_TN and bias is None and act is None and residual is None and colstats is None
                and not row_remap and not out_f32 and swg_ok(M, N, K, lda, ldb) and ldc % 4 == 0
                and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0):
            ws = torch.empty(int(_lib.fn("ddl_stream_wgrad_ws")(M, N)), dtype=torch.bfloat16, device=C.device)
            rc = _lib.fn("ddl_stream_wgrad")(A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(), ldc, M, N, K,
                                             int(accumulate), ws.data_ptr(), ws.numel(),
                                             _zero_page(C.device).data_ptr(), 0, _lib.stream())
            if rc != 0:
                raise RuntimeError(f"ddl_stream_wgrad(M={M}, N={N}, K={K}) failed: {rc}")
            return
        kind, s = _heuristic(mode, M, N, K, row_remap, lda, ldb)   # a cached choice outside its contract
    if kind == "duo" and mode == MODE_TN:
        if (bias is None and act is None and residual is None and colstats is None and not row_remap
                and C.dtype == torch.bfloat16 and duo_tn_ok(M, N, K, lda, ldb, ldc)
                and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0 and C.data_ptr() % 16 == 0):
            ws = torch.empty(s * M * N, dtype=torch.bfloat16, device=C.device) if s > 1 else None
            rc = _lib.fn("ddl_gemm_duo_tn")(A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(), ldc, M, N, K, s,
                                            int(accumulate), _lib.p(ws), 0 if ws is None else ws.numel(),
                                            _lib.stream())
            if rc < 0:
                raise RuntimeError(f"ddl_gemm_duo_tn(M={M}, N={N}, K={K}, splits={s}) failed: {rc}")
            return
        kind, s = _heuristic(mode, M, N, K, row_remap, lda, ldb)   # a cached choice outside its contract
    if kind == "duo":
        conv_c = None if conv_arr is None else int(conv_arr[3])
        if duo_ok(mode, M, N, K, lda, ldb, ldc, bias, act, aux, residual, colstats, row_remap, conv_c,
                  accumulate, C) and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0 and C.data_ptr() % 16 == 0:
            if bnb is not None:   # ACT_BNB side arguments (mask, mean, invstd), consumed by this launch
                _lib.fn("ddl_gemm_bnb")(_lib.p(bnb[0]), _lib.p(bnb[1]), _lib.p(bnb[2]))
            rc = _lib.fn("ddl_gemm_duo")(mode, A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(), ldc, M, N, K,
                                         _lib.p(bias), ACT[act], _lib.p(aux), _lib.p(residual), _lib.p(colstats),
                                         conv_arr, _lib.stream())
            if rc != 0:
                raise RuntimeError(f"ddl_gemm_duo(mode={mode}, M={M}, N={N}, K={K}) failed: {rc}")
            return
        kind, s = _heuristic(mode, M, N, K, row_remap, lda, ldb)   # a cached choice outside its contract
    if kind in ("wg", "wg2"):
        cw = mode == MODE_CONVW and conv_arr is not None and conv_arr[3] % 8 == 0
        wide = kind == "wg2"
        if ((mode == MODE_TN or cw) and bias is None and act is None and residual is None and colstats is None
                and not row_remap and wg_ok(M, N, K, lda, ldb, wide) and ldc % 4 == 0
                and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0):
            ws = torch.empty(max(1, s) * M * ldc, dtype=torch.float32, device=C.device)
            rc = _lib.fn("ddl_gemm_wgrad")(A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(), ldc, M, N, K, out_f32,
                                           s, ws.data_ptr(), ws.numel(), int(accumulate),
                                           conv_arr if cw else None, _zero_page(C.device).data_ptr(), int(wide),
                                           _lib.stream())
            if rc != 0:
                raise RuntimeError(f"ddl_gemm_wgrad(M={M}, N={N}, K={K}, splits={s}) failed: {rc}")
            return
        kind, s = _heuristic(mode, M, N, K, row_remap, lda, ldb)   # a cached choice outside its contract
    ws = torch.empty(s * M * (N if mode & TRANS_OUT else ldc), dtype=torch.float32, device=C.device) \
        if s > 1 else None
    args = (mode, A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(), ldc, M, N, K, _lib.p(bias), bias_bf16,
            ACT[act], _lib.p(aux), out_f32, s, _lib.p(ws), 0 if ws is None else ws.numel(), conv_arr,
            int(row_remap), _lib.p(residual), int(accumulate))
    cs = _lib.p(colstats)
    if bnb is not None:   # ACT_BNB side arguments (mask, mean, invstd), consumed by this launch
        _lib.fn("ddl_gemm_bnb")(_lib.p(bnb[0]), _lib.p(bnb[1]), _lib.p(bnb[2]))
    if kind in ("big", "big192"):
        if kind == "big192":
            args = (mode | N192,) + args[1:]
        rc = _lib.fn("ddl_gemm_big2")(*args, _zero_page(C.device).data_ptr(), cs, _lib.stream())
    elif kind == "narrow":
        rc = _lib.fn("ddl_gemm_n64")(*args, cs, _lib.stream())
    else:
        rc = _lib.fn("ddl_gemm")(*args, cs, _lib.stream())
    if rc != 0:
        raise RuntimeError(f"ddl_gemm[{kind}](mode={mode}, M={M}, N={N}, K={K}, splits={s}) failed: {rc}")


def _big_allowed(mode: int, K: int, lda: int = 8, ldb: int = 8) -> bool:
    # 16-byte LDS-DMA rows: K and both leading dimensions in whole 8-element chunks
    return not _force_small and mode != MODE_CONVW and K % 8 == 0 and K >= 64 and lda % 8 == 0 and ldb % 8 == 0


def _candidates(mode: int, M: int, N: int, K: int, row_remap: bool, lda: int, ldb: int, plain: bool = False,
                conv_c: Optional[int] = None):
    """(kernel, splits) variants worth timing for one GEMM shape: each kernel at
    no split, its heuristic split and half of it (split-K trades parallelism
    against fp32 partial-slab traffic, which the heuristic cannot price)."""
    out = []
    if _big_allowed(mode, K, lda, ldb):
        bs = 1 if row_remap else big_splits(M, N, K)
        out += [("big", s) for s in sorted({1, max(1, bs // 2), bs})]
    ps = 1 if row_remap else pick_splits(M, N, K)
    out += [("small", s) for s in sorted({1, max(1, ps // 2), ps})]
    if N <= 192 or N % 128 == 64:     # 128x64 tiles: no half-empty column tile
        ns = 1 if row_remap else pick_splits(M, 2 * N, K)   # 128x64 tiles = 128x128 tiles on 2N
        out += [("narrow", s) for s in sorted({1, max(1, ns // 2), ns})]
    if _WG and plain and wg_ok(M, N, K, lda, ldb) and (
            mode == MODE_TN or (mode == MODE_CONVW and conv_c is not None and conv_c % 8 == 0)):
        # weight-gradient kernel (gemm_big.hip gemm_wg_k): 4 waves on 256x128 tiles ("wg") and 8 waves on
        # 256x256 tiles ("wg2"); fp32 partials + reduce
        ws_ = big_splits(M, 2 * N, K)      # 256x128 tiles = 256x256 tiles on 2N
        out += [("wg", s) for s in sorted({max(1, ws_ // 2), ws_, 2 * ws_})]
        if _WG2 and N % 256 == 0:
            w2 = big_splits(M, N, K)
            out += [("wg2", s) for s in sorted({max(1, w2 // 2), w2, 2 * w2})]
    if _DUO and mode == MODE_TN and plain and not row_remap and duo_tn_ok(M, N, K, lda, ldb):
        # dual-workgroup kernel, k-outer A: bf16 partial tiles + one reduce (split 1: straight into C)
        ds = duo_tn_splits(M, N, K)
        out += [("duo", s) for s in sorted({max(1, ds // 2), ds, min(2 * ds, K // 32)})]
    if _SWG and mode == MODE_TN and plain and not row_remap and swg_ok(M, N, K, lda, ldb):
        # streaming weight gradient (stream_gemm.hip stream_wgrad_k): every workgroup owns the whole
        # M x N output over a range of K rows (no operand re-reads), bf16 partials + one reduce
        out.append(("swg", 1))
    if mode in (MODE_TN, MODE_CONVW) and plain and (M <= 192 or M % 128 == 64):
        ts = pick_splits(N, 2 * M, K)     # transposed: N' = M (output channels) on 64-wide tiles
        out += [("tnarrow", s) for s in sorted({1, max(1, ts // 2), ts})]
    if mode in (MODE_NT, MODE_NN) and not row_remap and _big_allowed(mode, K, lda, ldb) and N % 192 == 0 \
            and _DIRECT:
        # 256 x 192 tiles: whole rounds where 256-wide ones leave a partial one (N = 768: 192 -> 256 tiles
        # at M = 16384); register epilogue only (the caller drops it for the BatchNorm-backward epilogue)
        out += [("big192", 1)] if _BIG192 else []
    if _HYBRID and mode in (MODE_NT, MODE_NN) and not row_remap and _big_allowed(mode, K, lda, ldb):
        hy = hybrid_rows(M, N, K)
        if hy is not None:                # a partial last round of 256x256 tiles
            out += [("hybrid", s) for s in sorted({2, max(2, hy[1] // 2), hy[1]})]
    return out


_WG = os.environ.get("DDL_GEMM_WG", "1") != "0"   # tuner candidate "wg" (A/B: 0 = never)
# "wg2" (8 waves, 256x256 tiles) is opt-in: at two waves per SIMD its 128x64 wave tiles plus fragments
# exceed the 256-register budget and spill in the loop -- slower than both "wg" and the 256x256 kernel
# on every BERT-base weight gradient (profiles/tn_kinds_r04_wg2.log)
_WG2 = os.environ.get("DDL_GEMM_WG2", "0") == "1"


_SWG = os.environ.get("DDL_GEMM_SWG", "1") != "0"   # tuner candidate "swg" (A/B: 0 = never)


_DUO = os.environ.get("DDL_GEMM_DUO", "1") != "0"   # tuner candidate "duo" (A/B: 0 = never)


def duo_ok(mode: int, M: int, N: int, K: int, lda: int, ldb: int, ldc: int, bias, act, aux, residual, colstats,
           row_remap=False, conv_c=None, accumulate=False, C=None) -> bool:
    """Calls the dual-workgroup 256x128 kernel takes (gemm_duo.hip ddl_gemm_duo's contract): NT / NN
    bf16 GEMMs and implicit-GEMM convolutions (``conv_c``: the input channel count, % 32 == 0; no
    output row remap) with N % 128 == 0, K % 32 == 0, 8-element leading dimensions, operands under
    2 GB, and a bias / residual / GELU (+ pre-activation) / dGELU / BatchNorm-backward / column-
    statistics epilogue."""
    if mode not in (MODE_NT, MODE_NN, MODE_CONV) or row_remap or accumulate:
        return False
    if mode == MODE_CONV:
        if conv_c is None or conv_c % 32:
            return False
    elif conv_c is not None or lda % 8 or lda < K or M * lda * 2 >= 2 ** 31:
        return False
    if N % 128 or K % 32 or K <= 0 or ldb % 8 or ldc % 8 or ldc < N:
        return False
    if (ldb < N if mode == MODE_NN else ldb < K):
        return False
    if C is not None and C.dtype != torch.bfloat16:
        return False
    if bias is not None and bias.dtype != torch.bfloat16:
        return False
    if act is None:
        pass
    elif act == "gelu":
        if residual is not None or colstats is not None:
            return False
    elif act == "dgelu":
        if aux is None or bias is not None or residual is not None:
            return False
    elif act == "bnb":
        if aux is None or bias is not None or colstats is None or ldc != N:
            return False
    else:
        return False
    if (K if mode == MODE_NN else N) * ldb * 2 >= 2 ** 31 or M * ldc * 2 >= 2 ** 31:
        return False
    return True


def duo_tn_ok(M: int, N: int, K: int, lda: int, ldb: int, ldc: int = None) -> bool:
    """TN weight gradients the dual-workgroup kernel takes (ddl_gemm_duo_tn's contract)."""
    ldc = N if ldc is None else ldc
    return M % 256 == 0 and N % 128 == 0 and K % 32 == 0 and K > 0 and lda % 8 == 0 and ldb % 8 == 0 \
        and ldc % 8 == 0 and lda >= M and ldb >= N and ldc >= N and K * lda * 2 < 2 ** 31 \
        and K * ldb * 2 < 2 ** 31 and M * ldc * 2 < 2 ** 31


def duo_tn_splits(M: int, N: int, K: int) -> int:
    """Split-K count that fills two workgroups per CU with 256 x 128 (tile, split) blocks."""
    tiles = (M // 256) * (N // 128)
    return max(1, min((K // 32) // 4, (2 * NUM_CU) // max(tiles, 1)))


def swg_ok(M: int, N: int, K: int, lda: int, ldb: int) -> bool:
    """Shapes the streaming weight-gradient kernel takes (ddl_stream_wgrad's contract): M, N in
    {64, 128, 256, 512} with M * N <= 64 Ki (the output in registers), a long reduction."""
    return M in (64, 128, 256, 512) and N in (64, 128, 256, 512) and M * N <= 65536 and K >= 8192 \
        and lda % 8 == 0 and ldb % 8 == 0 and lda >= M and ldb >= N


def wg_ok(M: int, N: int, K: int, lda: int, ldb: int, wide: bool = False) -> bool:
    """Shapes the weight-gradient kernel takes (ddl_gemm_wgrad's contract: 256x128 tiles, or 256x256
    for the 8-wave ``wide`` variant "wg2")."""
    return M % 256 == 0 and N % (256 if wide else 128) == 0 and K % 128 == 0 and K > 0 and lda % 8 == 0 \
        and ldb % 8 == 0


def _heuristic(mode: int, M: int, N: int, K: int, row_remap: bool, lda: int, ldb: int):
    if use_big(mode, M, N, K) and _big_allowed(mode, K, lda, ldb):
        return ("big", 1 if row_remap else big_splits(M, N, K))
    return ("small", 1 if row_remap else pick_splits(M, N, K))


# Measured kernel choice per GEMM signature (like cudnn.benchmark): the first call
# of a shape times every candidate into scratch outputs and caches the fastest;
# the bench's warmup steps absorb this.  DDL_GEMM_TUNE=0 uses the static heuristic.
_tuned: dict = {}
# candidate timings behind each tuned choice (ms per call, this process): what
# agree_across_ranks() pools so every data-parallel rank runs the same kernel plan
_timings: dict = {}
_NARROW_STATS = os.environ.get("DDL_TUNE_NARROW_STATS", "0") != "0"   # same-box A/B neutral: off
_TUNE = os.environ.get("DDL_GEMM_TUNE", "1") != "0"
# DDL_GEMM_PREFER=kind[:factor]: take `kind` when it is within `factor` of the fastest candidate.  Default
# "swg:1.3": the cold-cache timing over-prices the streaming weight-gradient kernel (it streams its
# operands once, in-model often from the Infinity Cache the producing pass just filled): ResNet-50
# same-box alternating, backward 14.61-14.63 vs 14.73-14.78 ms, 11,676-11,739 vs 11,637-11,693 img/s
_PREFER = os.environ.get("DDL_GEMM_PREFER", "swg:1.3")
_TUNE_ROUNDS = max(1, int(os.environ.get("DDL_GEMM_TUNE_ROUNDS", "5")))   # interleaved timing rounds per candidate
_TUNE_COLD = os.environ.get("DDL_GEMM_TUNE_COLD", "1") != "0"             # time candidates from evicted caches
# in-model tuning during warm-up: "1" always, "0" never, unset: the caller's default (the trainer turns it
# on for transformer models, whose GEMM operands stay cache-resident in-model -- see online_tuning)
_ONLINE_ENV = os.environ.get("DDL_GEMM_TUNE_ONLINE")
_ONLINE = _ONLINE_ENV == "1"
# optional persistent cache (JSON): later processes skip the timing runs
_CACHE_PATH = os.environ.get("DDL_GEMM_TUNE_CACHE", "")

# ------------------------------------------------------------------ committed kernel plan table
# A reproducible plan by default (SURVEY §5.4-style determinism for the GEMM plan): ``gemm_plans.json``
# holds measured (kernel, splits) choices per GEMM signature, keyed by GPU architecture and by the
# hash of the GEMM kernel sources the library was built from (``csrc/build.py`` gemm_src_hash).  A
# signature in the table runs its committed plan in every process -- whatever the warm-up count,
# whichever entry point (bench.py, the train() presets, notebooks) -- so two fresh processes run the
# same kernels; only a miss is tuned (isolated / in-model tuner, as before).  The table is refreshed
# from tuning runs by ``scripts/make_plan_table.py``.  DDL_GEMM_PLAN_TABLE=0 disables it, or names
# another table file.  Precedence: an explicit DDL_GEMM_TUNE_CACHE entry, then the table, then tuning.
_TABLE_ENV = os.environ.get("DDL_GEMM_PLAN_TABLE", "1")
_TABLE_PATH = _TABLE_ENV if _TABLE_ENV not in ("0", "1", "") else \
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_plans.json")
_table: Optional[dict] = None            # key -> (kind, splits), loaded on first use
_table_info = {"path": _TABLE_PATH if _TABLE_ENV != "0" else None, "arch": None, "gemm_src_hash": None,
               "status": "not loaded", "entries": 0}
_table_hits: set = set()
_table_misses: set = set()
_used: Optional[set] = None              # signatures looked up since plan_usage() started


def _device_arch() -> str:
    try:
        return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
    except Exception:   # noqa: BLE001 -- no GPU: no table
        return ""


def load_plan_table() -> dict:
    """The committed plans for this GPU architecture and GEMM-kernel build ({} when the table is
    disabled, missing, or was tuned against other kernel sources / another architecture)."""
    global _table
    if _table is not None:
        return _table
    _table = {}
    if _TABLE_ENV == "0":
        _table_info["status"] = "disabled"
        return _table
    arch, src = _device_arch(), _lib.gemm_src_hash()
    _table_info.update(arch=arch, gemm_src_hash=src)
    try:
        with open(_TABLE_PATH) as f:
            doc = json.load(f)
    except (OSError, ValueError) as e:
        _table_info["status"] = f"unreadable ({type(e).__name__})"
        return _table
    ent = doc.get(arch)
    if not ent:
        _table_info["status"] = f"no plans for {arch or 'this device'}"
    elif src is None or ent.get("gemm_src_hash") != src:
        _table_info["status"] = f"stale (tuned for GEMM sources {ent.get('gemm_src_hash')}, library has {src})"
    else:
        _table = {k: (v[0], int(v[1])) for k, v in ent.get("plans", {}).items()}
        _table_info.update(status="loaded", entries=len(_table))
    return _table


def plan_stats() -> dict:
    """Where this process's GEMM plan came from: ``source`` = "table" (every signature from the
    committed table), "table+tuned" (some tuned: ``misses`` counts them) or "tuned"."""
    hits, miss = len(_table_hits), len(_table_misses)
    src = "table" if hits and not miss else "table+tuned" if hits else "tuned"
    return dict(_table_info, source=src, table_hits=hits, misses=miss)


@contextlib.contextmanager
def plan_usage():
    """Collect the signatures looked up inside the block: ``with plan_usage() as used: ...``."""
    global _used
    prev, _used = _used, set()
    try:
        yield _used
    finally:
        _used = prev


def lookup_choice(key: str):
    """A non-GEMM kernel choice (e.g. the strided-conv dgrad path) from this process's tuning / the tune
    cache, else from the committed plan table; None = not planned (the caller tunes and records it)."""
    if _used is not None:
        _used.add(key)
    v = _tuned.get(key)
    if v is None:
        v = load_plan_table().get(key)
        (_table_hits if v is not None else _table_misses).add(key)
    return v


def record_choice(key: str, value) -> None:
    """Remember a choice tuned in this process (and in DDL_GEMM_TUNE_CACHE, so tuning runs feed the table)."""
    _tuned[key] = tuple(value)
    _save_cache()


def current_plan(keys) -> dict:
    """(kernel, splits) of each signature in ``keys`` as this process runs it."""
    tab = load_plan_table()
    out = {}
    for k in keys:
        v = _tuned.get(k) or tab.get(k)
        if v is not None:
            out[k] = v
    return out


def _load_cache() -> None:
    if not _CACHE_PATH or not os.path.exists(_CACHE_PATH):
        return
    try:
        with open(_CACHE_PATH) as f:
            for k, v in json.load(f).items():
                _tuned[k] = tuple(v)
    except (OSError, ValueError):
        pass


def _save_cache() -> None:
    if not _CACHE_PATH:
        return
    tmp = f"{_CACHE_PATH}.{os.getpid()}.tmp"
    try:
        with open(tmp, "w") as f:
            json.dump({k: list(v) for k, v in _tuned.items()}, f)
        os.replace(tmp, _CACHE_PATH)
    except OSError:
        pass


_load_cache()


def tuned_choices() -> dict:
    return dict(_tuned)


def agree_across_ranks(group=None) -> int:
    """Make every rank of ``group`` run the SAME kernel for every tuned GEMM signature.

    Each rank times candidates on its own GPU during warm-up; independent choices can
    differ (timer noise on close calls) and the slowest rank's plan then gates every
    data-parallel step.  This all-gathers the per-candidate timings (a small object
    collective on the host group -- call it between steps, never inside backward),
    sums them over the ranks that tuned the signature and sets the argmin everywhere.
    All ranks compute the same answer from the same gathered data.  Returns how many
    signatures had a rank whose choice changed -- the SAME number on every rank, so a
    caller that re-runs a warm-up step when it is > 0 (a changed plan may route later
    GEMMs through signatures not tuned yet) does so on every rank or on none (a per-rank
    count let one rank run an extra step alone: a collective deadlock)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return 0
    mine = {"timings": {k: {f"{kind}:{s}": t for (kind, s), t in v.items()} for k, v in _timings.items()},
            "tuned": {k: f"{v[0]}:{v[1]}" for k, v in _tuned.items()}}
    gathered = [None] * dist.get_world_size(group)
    dist.all_gather_object(gathered, mine, group=group)
    keys = set()
    for g in gathered:
        keys.update(g["timings"].keys())
    changed = 0
    for key in sorted(keys):
        tot: dict = {}
        for g in gathered:
            for c, t in g["timings"].get(key, {}).items():
                tot.setdefault(c, []).append(t)
        n = max(len(v) for v in tot.values())
        # only candidates every tuning rank timed compete (the same list on each rank)
        best = min((sum(v), c) for c, v in tot.items() if len(v) == n)[1]
        if any(g["tuned"].get(key, best) != best for g in gathered):
            changed += 1
        kind, s = best.split(":")
        _tuned[key] = (kind, int(s))
    _save_cache()
    return changed


_flush_bufs: dict = {}


def _flush_buf(device) -> torch.Tensor:
    """A 640 MB scratch buffer whose fill evicts the L2s and the 256 MB Infinity Cache."""
    b = _flush_bufs.get(device)
    if b is None:
        b = _flush_bufs[device] = torch.empty(640 << 20, dtype=torch.uint8, device=device)
    return b


def release_tuning_buffers() -> None:
    """Drop the tuner's cache-flush buffers (640 MB each): called once the warm-up has tuned every
    signature, so that HBM returns to the allocator for the training step (a signature first seen
    later re-creates its buffer on demand)."""
    _flush_bufs.clear()


def _time_runs(run, reps: int, cold: bool = False) -> float:
    """Milliseconds per call over ``reps`` launches, in DEVICE time.

    A spin kernel (``torch.cuda._sleep``) goes first so the host has queued every launch
    before the first timing event is reached: otherwise a kernel shorter than the ~40-60 us
    the Python launch path takes is timed at the HOST's launch rate -- the same for every
    candidate -- and the tuner's pick among fast kernels was noise.  ``cold``: every launch is
    preceded by a cache-evicting fill and timed alone (events around the launch only): a
    training step's GEMM reads operands that were written long before (saved activations,
    weights), and with every operand cache-hot the 128x128 kernels won the weight-gradient
    GEMMs they lose in the model (BERT-base backward +1.7 ms/step when they were picked)."""
    if hasattr(torch.cuda, "_sleep"):
        torch.cuda._sleep(int(min(4e8, (4.0e5 if cold else 2.5e5) * (reps + 1))))   # ~120-190 us host time per launch
    if not cold:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps
    buf = _flush_buf(torch.cuda.current_device())
    evs = []
    for _ in range(reps):
        buf.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        evs.append((a, b))
    evs[-1][1].synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / reps


def _tune_candidates(mode, M, N, K, lda, ldb, bias, act, aux, row_remap, residual, colstats, conv_c=None):
    """The (kernel, splits) candidates a call of this signature can run (``conv_c``: a convolution's
    input channel count)."""
    plain = bias is None and act is None and residual is None and aux is None and not row_remap
    cands = _candidates(mode, M, N, K, row_remap, lda, ldb, plain, conv_c)
    if act not in (None, "relu", "gelu", "dgelu") or (act == "dgelu" and aux is None):
        cands = [c for c in cands if c[0] != "big192"]     # LDS-staged epilogue: 256-wide tiles only
    if _DUO and duo_ok(mode, M, N, K, lda, ldb, N, bias, act, aux, residual, colstats, row_remap, conv_c):
        cands.append(("duo", 1))
    if act == "dgelu" and colstats is not None:
        # dGELU column sums: register epilogues only (256x256 / 256x192 / dual-workgroup kernels)
        cands = [c for c in cands if c[0] in ("big", "big192", "duo")]
    if colstats is not None:   # statistics epilogue: whole-K tiles only
        cands = [c for c in cands if c[1] == 1 and not c[0].startswith("t")]
        # 128x64 tiles (three blocks per CU) for the epilogue-heavy statistics / BN-backward
        # tiles even where N is a multiple of 128 (more blocks in flight per CU)
        if _NARROW_STATS and N % 64 == 0 and ("narrow", 1) not in cands:
            cands.append(("narrow", 1))
    return cands


def _tune(key, mode, A, lda, B, ldb, C, ldc, M, N, K, bias, act, aux, conv_arr, row_remap, residual,
          colstats=None, bnb=None):
    cands = _tune_candidates(mode, M, N, K, lda, ldb, bias, act, aux, row_remap, residual, colstats,
                             None if conv_arr is None else int(conv_arr[3]))
    cs_s = torch.empty_like(colstats) if colstats is not None else None
    if len(cands) == 1:
        _timings[key] = {cands[0]: 0.0}
        return cands[0]
    Cs = torch.empty_like(C)
    aux_s = aux
    if aux is not None and act in ("gelu", "relu", "tanh"):   # aux is an output for these
        aux_s = torch.empty_like(aux)
    runs = []
    for kind, s in cands:
        run = lambda kind=kind, s=s: _launch(kind, s, mode, A, lda, B, ldb, Cs, ldc, M, N, K, bias, act,  # noqa: E731
                                             aux_s, conv_arr, row_remap, residual, False, cs_s, bnb)
        run()                              # first launch: code object load, caches
        runs.append(run)
    # Candidates are timed INTERLEAVED over rounds and ranked by their median: a one-shot
    # sequential timing let clock / cache drift between candidates decide close calls, so
    # fresh processes could tune different plans for the same shapes.
    est = [_time_runs(r, 1) for r in runs]
    reps = max(2, min(8, int(0.3 / max(min(est), 1e-3))))
    rounds = [[] for _ in runs]
    for _ in range(_TUNE_ROUNDS):
        for ci, r in enumerate(runs):
            rounds[ci].append(_time_runs(r, reps, cold=_TUNE_COLD))
    med = [sorted(v)[len(v) // 2] for v in rounds]
    _timings[key] = {c: t for c, t in zip(cands, med)}
    best = min(range(len(cands)), key=lambda i: med[i])
    fastest = best
    for pref in filter(None, _PREFER.split(",")):
        # DDL_GEMM_PREFER=kind[:factor],...: the first listed kind within `factor` of the fastest candidate
        kind, _, f = pref.partition(":")
        near = [i for i, c in enumerate(cands) if c[0] == kind and med[i] <= med[fastest] * float(f or "1.5")]
        if near:
            best = min(near, key=lambda i: med[i])
            break
    return cands[best]


# ------------------------------------------------------------------ in-model (online) tuning
# Opt-in (DDL_GEMM_TUNE_ONLINE=1): during a trainer's warm-up steps an untuned signature cycles
# through its candidates on its REAL calls (every layer's call is a sample, timed with events on the
# compute stream, read back once per step) and keeps the one with the lowest median in-model time.
# It was built when the isolated tuner kept the BERT-base weight-gradient GEMMs on the 128x128
# kernel; the cause turned out to be register spills in the 256x256 kernel's TN loop
# (profiles/gemm_spills_r04.md).  Round 5: the isolated tuner times every candidate on COLD caches,
# which is right for ResNet's 100-411 MB activations but not for transformer GEMMs, whose operands stay
# in the 256 MB last-level cache in-model: in-model tuning picks plans worth +2.2 % on BERT-base
# (and -0.7 % on ResNet-50; profiles/online_tune_ab.log).  The trainer therefore turns it on for
# transformer models (default=True below) and leaves CNNs on the isolated tuner.  The price: warm-up
# steps cycle through candidates with different split-K summation orders, so those steps round
# differently than in a process whose tune cache is already warm.
_online_active = False
_online_max_bytes = float("inf")   # signatures touching more operand + output bytes stay on the isolated tuner
_online: dict = {}          # key -> {"cands": [...], "n": calls, "pending": [(cand, e0, e1)], "samples": {}}
_online_last = None         # (key, cand) of the call _choose just routed online
_online_count = {"tuned": 0, "samples": 0}


def online_stats() -> dict:
    """How many signatures in-model tuning committed, from how many timed calls (this process)."""
    return dict(_online_count)


@contextlib.contextmanager
def online_tuning(enabled: bool = True, default: bool = False, max_mb: float = float("inf")):
    """Tune untuned GEMM signatures from their in-model calls inside the block (the trainer's
    warm-up steps); call :func:`online_collect` after each step.  On exit every signature seen
    gets its in-model argmin (:func:`online_finish`).  ``default``: whether to tune in-model when
    DDL_GEMM_TUNE_ONLINE is unset; ``max_mb``: only signatures whose operands + output stay under
    it (cache-resident in-model) are tuned in-model, the others on the isolated cold-cache tuner."""
    global _online_active, _online_max_bytes
    prev, prev_max = _online_active, _online_max_bytes
    want = _ONLINE or (_ONLINE_ENV is None and default)
    _online_active = bool(enabled) and _TUNE and want and torch.cuda.is_available()
    _online_max_bytes = max_mb * 2 ** 20
    try:
        yield
    finally:
        if _online_active:
            online_finish()
        _online_active, _online_max_bytes = prev, prev_max


def online_collect() -> None:
    """Read back the events of the calls timed since the last collect (one host sync)."""
    pend = [(st, c, a, b) for st in _online.values() for c, a, b in st["pending"]]
    if not pend:
        return
    pend[-1][3].synchronize()
    torch.cuda.synchronize()
    for st, c, a, b in pend:
        st["samples"].setdefault(c, []).append(a.elapsed_time(b))
    for st in _online.values():
        st["pending"] = []


def online_finish() -> int:
    """Commit the in-model choice of every signature tuned online; returns how many."""
    online_collect()
    done = 0
    for key, st in list(_online.items()):
        med = {c: sorted(v)[len(v) // 2] for c, v in st["samples"].items() if v}
        if med:
            _timings[key] = med
            _tuned[key] = min(med, key=med.get)
            done += 1
            _online_count["samples"] += sum(len(v) for v in st["samples"].values())
        del _online[key]
    _online_count["tuned"] += done
    if done:
        _save_cache()
    return done


def _choose(mode, A, lda, B, ldb, C, ldc, M, N, K, bias, act, aux, splits, conv, conv_arr, row_remap, residual,
            kernel, colstats, bnb=None, online_ok: bool = False):
    """(kernel kind, splits) for one GEMM call: forced, explicit, tuned (cached) or heuristic."""
    kernel = kernel or _forced
    if kernel == "big192" and not (mode in (MODE_NT, MODE_NN) and not row_remap and _DIRECT and
                                   _big_allowed(mode, K, lda, ldb) and act in (None, "relu", "gelu", "dgelu")
                                   and not (act == "dgelu" and aux is None)):
        kernel = "big"                    # 192-wide tiles: NT / NN with a register epilogue only
    if kernel is not None:
        if kernel == "big" and not _big_allowed(mode, K, lda, ldb):
            kernel = "small"              # no 256x256 variant for these
        hy = hybrid_rows(M, N, K) if kernel == "hybrid" and mode in (MODE_NT, MODE_NN) and not row_remap \
            and colstats is None and _big_allowed(mode, K, lda, ldb) else None
        if kernel == "hybrid":
            kernel = "big" if hy is None else kernel     # no partial round: the plain launch
        if kernel == "big192":
            choice = ("big192", 1)
        elif hy is not None:
            choice = ("hybrid", max(2, splits or hy[1]))
        elif kernel == "big":
            choice = ("big", 1 if row_remap else (splits or big_splits(M, N, K)))
        elif kernel == "narrow":
            choice = ("narrow", 1 if row_remap else pick_splits(M, 2 * N, K, splits))
        elif kernel in ("wg", "wg2") \
                and (mode == MODE_TN or (mode == MODE_CONVW and conv is not None and conv[3] % 8 == 0)) \
                and bias is None and act is None and residual is None and not row_remap and colstats is None \
                and wg_ok(M, N, K, lda, ldb, kernel == "wg2"):
            choice = (kernel, splits or big_splits(M, N, K))
        elif kernel == "duo" and mode == MODE_TN and bias is None and act is None and residual is None \
                and colstats is None and not row_remap and duo_tn_ok(M, N, K, lda, ldb, ldc):
            choice = ("duo", splits or duo_tn_splits(M, N, K))
        elif kernel == "duo" and duo_ok(mode, M, N, K, lda, ldb, ldc, bias, act, aux, residual, colstats, row_remap,
                                        None if conv is None else int(conv[3]), False, C):
            choice = ("duo", 1)
        elif kernel == "tnarrow" and mode in (MODE_TN, MODE_CONVW) and bias is None and act is None \
                and residual is None and not row_remap and colstats is None:
            choice = ("tnarrow", pick_splits(N, 2 * M, K, splits))
        else:
            choice = ("small", 1 if row_remap else pick_splits(M, N, K, splits))
        if colstats is not None:
            choice = ("small" if choice[0] == "tnarrow" else choice[0], 1)
    elif splits is not None:                       # explicit request: 128x128 kernel with that split
        choice = ("small", 1 if row_remap else pick_splits(M, N, K, splits))
    elif _TUNE and not _force_small and C.is_cuda:
        key = f"{mode}|{M}|{N}|{K}|{lda}|{ldb}|{ldc}|{tuple(conv) if conv is not None else ''}|{int(row_remap)}|" \
              f"{act}|{C.dtype}|{int(bias is not None)}|{int(colstats is not None)}|{int(residual is not None)}"
        if _used is not None:
            _used.add(key)
        choice = _tuned.get(key)
        if choice is None:
            choice = load_plan_table().get(key)
            if choice is not None:
                _table_hits.add(key)
            else:
                _table_misses.add(key)
        if choice is None and online_ok and _online_active and not torch.cuda.is_current_stream_capturing() \
                and (A.numel() + B.numel() + C.numel()) * C.element_size() <= _online_max_bytes:
            global _online_last
            st = _online.get(key)
            if st is None:
                cands = _tune_candidates(mode, M, N, K, lda, ldb, bias, act, aux, row_remap, residual, colstats,
                                         None if conv is None else int(conv[3]))
                st = _online[key] = {"cands": cands, "n": 0, "pending": [], "samples": {}}
            choice = st["cands"][st["n"] % len(st["cands"])]
            st["n"] += 1
            _online_last = (key, choice)
        if choice is None:
            if torch.cuda.is_current_stream_capturing():   # cannot time inside a graph capture
                choice = _heuristic(mode, M, N, K, row_remap, lda, ldb)
            else:
                choice = _tune(key, mode, A, lda, B, ldb, C, ldc, M, N, K, bias, act, aux, conv_arr, row_remap,
                               residual, colstats, bnb)
                _tuned[key] = choice
                _save_cache()
    else:
        choice = _heuristic(mode, M, N, K, row_remap, lda, ldb)
    if colstats is not None and (choice[1] != 1 or choice[0].startswith("t")):
        choice = (choice[0] if choice[0] in ("big", "big192", "duo") else "small", 1)
        if act == "dgelu" and choice[0] == "small" and _big_allowed(mode, K, lda, ldb):
            choice = ("big", 1)        # dGELU column sums: register epilogues only
    return choice


def plan(mode: int, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int, C: torch.Tensor, ldc: int,
         M: int, N: int, K: int, conv: Optional[Sequence[int]] = None, residual: Optional[torch.Tensor] = None,
         full: bool = False):
    """The kernel kind (``full``: the (kind, splits) pair) a plain call of this signature
    runs, tuning it now if needed."""
    conv_arr = None if conv is None else (ctypes.c_int * len(conv))(*[int(v) for v in conv])
    ch = _choose(mode, A, lda, B, ldb, C, ldc, M, N, K, None, None, None, None, conv, conv_arr, False,
                 residual, None, None)
    return ch if full else ch[0]


def gemm(mode: int, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int, C: torch.Tensor, ldc: int,
         M: int, N: int, K: int, bias: Optional[torch.Tensor] = None, act: Optional[str] = None,
         aux: Optional[torch.Tensor] = None, splits: Optional[int] = None,
         conv: Optional[Sequence[int]] = None, row_remap: bool = False,
         residual: Optional[torch.Tensor] = None, accumulate: bool = False,
         kernel: Optional[str] = None, colstats: Optional[torch.Tensor] = None, bnb=None):
    """C = op(A) op(B) (+ epilogue).  ``kernel`` forces "big" (256x256), "small" (128x128),
    "narrow" (128x64), "tnarrow" (weight gradient computed transposed on 128x64 tiles), "big192"
    (256x192 tiles of the 256x256 kernel: NT / NN, register epilogue) or
    "hybrid" (256x256 tiles, the rows past the last whole round split-K: ``hybrid_rows``) or "wg" (TN weight
    gradients on the 4-wave 256x256 kernel, fp32 partials + reduce: ``wg_ok`` shapes).  Every
    kind is a hand-written kernel of this library (no vendor GEMM library is ever called).

    ``colstats`` (fp32, >= ceil(M/128) * 2N elements): the epilogue also writes BatchNorm
    statistics partials of the bf16 output; the function then returns the number of
    partial rows written (one per M-tile).  Otherwise it returns ``C``.

    ``act="bnb"`` with ``bnb=(relu_mask or None, mean, invstd)`` and ``aux`` = the BatchNorm's
    input: the BatchNorm backward's reduction in the epilogue -- ``C`` receives
    dz = (result + residual) * mask and ``colstats`` rows [sum dz | sum dz * xhat].
    """
    conv_arr = None
    if conv is not None:
        conv_arr = (ctypes.c_int * len(conv))(*[int(v) for v in conv])
    global _online_last
    _online_last = None
    choice = _choose(mode, A, lda, B, ldb, C, ldc, M, N, K, bias, act, aux, splits, conv, conv_arr, row_remap,
                     residual, kernel, colstats, bnb, online_ok=True)
    online = _online_last
    _online_last = None
    if _trace is not None or online is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _launch(choice[0], choice[1], mode, A, lda, B, ldb, C, ldc, M, N, K, bias, act, aux, conv_arr, row_remap,
            residual, accumulate, colstats, bnb)
    if online is not None:
        e1.record()
        _online[online[0]]["pending"].append((online[1], e0, e1))
    if _trace is not None:
        e1.record()
        _trace.append(((mode, M, N, K, tuple(conv) if conv is not None else None, act, bias is not None,
                        residual is not None, colstats is not None, accumulate), choice, e0, e1))
    if colstats is not None:
        # one partial row per 128 output rows (256x256 tiles: one per wave row)
        return 2 * -(-M // 256) if choice[0] in ("big", "big192", "duo") else -(-M // 128)
    return C


def stats_rows_max(M: int) -> int:
    """Partial-row capacity a ``colstats`` buffer needs: one row per 128 output rows
    (128-row tiles), or two per 256-row tile of the large kernel."""
    return max(-(-M // 128), 2 * -(-M // 256))
