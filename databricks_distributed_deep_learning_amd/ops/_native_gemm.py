"""Thin wrapper over ``ddl_gemm`` (csrc/kernels/gemm.hip): modes, split-K policy, workspace."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from . import _lib
from ._lib import I, L, P

_lib.register({"ddl_gemm": [I, P, L, P, L, P, L, I, I, I, P, I, I, P, I, I, P, L, P, I, P, I, P],
               "ddl_gemm_big2": [I, P, L, P, L, P, L, I, I, I, P, I, I, P, I, I, P, L, P, I, P, I, P, P]})

MODE_NT, MODE_NN, MODE_TN, MODE_CONV, MODE_CONVW = 0, 1, 2, 3, 4
ACT = {None: 0, "gelu": 1, "relu": 2, "tanh": 3, "dgelu": 4}
BM = BN = 128
BK = 64
NUM_CU = 256
_force_small = False
_zero_pages = {}


def set_big_gemm(enabled: bool) -> None:
    """Route GEMMs to the 256x256 8-phase kernel (True, default) or the 128x128 one."""
    global _force_small
    _force_small = not enabled


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
    tiles = (-(-M // 256)) * (-(-N // 256))
    nk = -(-K // BK)
    if tiles >= 200:
        return 1
    return max(1, min(-(-NUM_CU // tiles), nk // 4))


def pick_splits(M: int, N: int, K: int, force: Optional[int] = None) -> int:
    """Split-K only when the tile grid cannot fill the chip; each split keeps >= 8 K-steps."""
    if force is not None:
        return max(1, force)
    tiles = -(-M // BM) * -(-N // BN)
    nk = -(-K // BK)
    if tiles >= NUM_CU or nk < 16:
        return 1
    return max(1, min(-(-2 * NUM_CU // tiles), nk // 8))


def gemm(mode: int, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int, C: torch.Tensor, ldc: int,
         M: int, N: int, K: int, bias: Optional[torch.Tensor] = None, act: Optional[str] = None,
         aux: Optional[torch.Tensor] = None, splits: Optional[int] = None,
         conv: Optional[Sequence[int]] = None, row_remap: bool = False,
         residual: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    conv_arr = None
    if conv is not None:
        conv_arr = (ctypes.c_int * len(conv))(*[int(v) for v in conv])
    bias_bf16 = 1 if (bias is not None and bias.dtype == torch.bfloat16) else 0
    out_f32 = 1 if C.dtype == torch.float32 else 0
    if splits is None and use_big(mode, M, N, K):
        s = 1 if row_remap else big_splits(M, N, K)
        ws = torch.empty(s * M * ldc, dtype=torch.float32, device=C.device) if s > 1 else None
        rc = _lib.fn("ddl_gemm_big2")(mode, A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(), ldc, M, N, K,
                                      _lib.p(bias), bias_bf16, ACT[act], _lib.p(aux), out_f32, s, _lib.p(ws),
                                      0 if ws is None else ws.numel(), conv_arr, int(row_remap),
                                      _lib.p(residual), int(accumulate), _zero_page(C.device).data_ptr(),
                                      _lib.stream())
        if rc != 0:
            raise RuntimeError(f"ddl_gemm_big2(mode={mode}, M={M}, N={N}, K={K}) failed: {rc}")
        return C
    s = 1 if row_remap else pick_splits(M, N, K, splits)
    ws = None
    if s > 1:
        ws = torch.empty(s * M * ldc, dtype=torch.float32, device=C.device)
    rc = _lib.fn("ddl_gemm")(mode, A.data_ptr(), lda, B.data_ptr(), ldb, C.data_ptr(), ldc, M, N, K,
                             _lib.p(bias), bias_bf16, ACT[act], _lib.p(aux), out_f32, s, _lib.p(ws),
                             0 if ws is None else ws.numel(), conv_arr, int(row_remap), _lib.p(residual),
                             int(accumulate), _lib.stream())
    if rc != 0:
        raise RuntimeError(f"ddl_gemm(mode={mode}, M={M}, N={N}, K={K}) failed: {rc}")
    return C
