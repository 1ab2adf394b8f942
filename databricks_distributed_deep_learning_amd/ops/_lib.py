"""Loader for the in-tree native kernel library (``libddl_kernels.so``).

The HIP kernels in ``csrc/kernels/*.hip`` are compiled by ``csrc/build.py``
(``hipcc --offload-arch=gfx950``) into one shared object with a plain C ABI:
every launcher takes raw device pointers, shapes and a ``hipStream_t``.  We load
it with ctypes *after* ``import torch`` so it binds to the HIP runtime PyTorch
already loaded (same SONAME ``libamdhip64.so.7``) and launches on PyTorch's
current stream — so the kernels are stream-ordered with ATen work and can be
captured into hipGraphs.

Policy (``DDL_NATIVE`` env or ``set_mode``):
  * ``auto`` (default): GPU tensors use the HIP kernels; if the library is
    missing on a GPU box we FAIL LOUDLY rather than silently fall back.
  * ``off``: stock PyTorch ops everywhere (the baseline arm of the benchmark).
  * CPU tensors always use the PyTorch reference implementations.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DDL_NATIVE_LIB: load another build of the library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("DDL_NATIVE_LIB") or os.path.join(_PKG_DIR, "_native", "libddl_kernels.so")

_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None
_mode = os.environ.get("DDL_NATIVE", "auto").lower()


class NativeUnavailable(RuntimeError):
    pass


def set_mode(mode: str) -> None:
    global _mode
    if mode not in ("auto", "on", "off"):
        raise ValueError(mode)
    _mode = mode


def mode() -> str:
    return _mode


def load() -> Optional[ctypes.CDLL]:
    global _lib, _load_error
    if _lib is not None or _load_error is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        _load_error = f"{LIB_PATH} not built (run `python csrc/build.py`)"
        return None
    try:
        _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        _load_error = str(e)
        return None
    return _lib


def gemm_src_hash() -> Optional[str]:
    """Hash of the GEMM kernel sources the loaded library was built from (``csrc/build.py``
    ``gemm_src_hash``), or None for a library built before it was recorded."""
    lib = load()
    if lib is None:
        return None
    try:
        fn = lib.ddl_gemm_src_hash
    except AttributeError:
        return None
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    return fn().decode()


def available() -> bool:
    return load() is not None


def load_error() -> Optional[str]:
    load()
    return _load_error


def use_native(*tensors: torch.Tensor) -> bool:
    """True when these (GPU) tensors should go through the HIP kernels."""
    if _mode == "off":
        return False
    if not all(t is None or t.is_cuda for t in tensors):
        return False
    if load() is None:
        raise NativeUnavailable(
            f"HIP kernel library unavailable on a GPU run: {_load_error}. "
            "Build it with `python csrc/build.py` or set DDL_NATIVE=off for stock PyTorch ops.")
    return True


def get() -> ctypes.CDLL:
    lib = load()
    if lib is None:
        raise NativeUnavailable(_load_error)
    return lib


def stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"native kernel {what} failed with HIP error {rc}")


# ------------------------------------------------------------------ signatures
P, I, L, F, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_uint64
_SIGS = {
    # norm.hip
    "ddl_bn_stats_nblk": [L, I],
    "ddl_bn_bwd_nblk": [L, I],
    "ddl_bn_rows_sum": [P, I, I, P, P, P],
    "ddl_rows_sum_sink": [I, P, I, I, I, P, I, P, P],
    "ddl_bn_stats_partials": [I, P, L, I, P, P],
    "ddl_bn_bwd_partials": [I, P, P, P, P, P, L, I, I, P, P],
    "ddl_bn_bwd_finish": [I, P, P, P, P, P, P, L, L, I, I, P, P, P, P, P, P, P, I, P],
    "ddl_bn_bwd_from_partials": [I, P, I, P, L, P, P, P, P, P, L, I, P, P, P, P, P, I, P],
    "ddl_bn_partials_ws": [I, I],
    "ddl_bn_fwd_train": [I, P, L, I, P, P, P, P, F, F, P, P, P, P, P, P],
    "ddl_bn_eval_coeffs": [I, I, P, P, P, P, F, P, P, P],
    "ddl_bn_apply": [I, P, P, P, P, P, L, I, I, P, P],
    "ddl_bn_apply2": [I, P, P, P, P, P, P, P, L, I, I, P, P],
    "ddl_bn_relu_maxpool": [I, P, P, P, P, P, P, I, I, I, I, I, I, P],
    "ddl_bn_bwd_pool_nblk": [],
    "ddl_bn_bwd_pool": [I, P, P, P, P, P, P, P, I, I, I, I, I, I, P, P, P, P, P, I, P],
    "ddl_bn_fwd_from_partials": [I, P, I, L, I, P, P, P, P, F, F, P, P, P, P, P, L],
    "ddl_conv_w_dgrad": [P, P, I, I, I, I, I, I, P, P, P],
    "ddl_conv_w_dgrad_batch": [P, P, I, P],
    "ddl_gelu_bwd_colsum": [I, P, P, P, L, I, P, P, I, I, P],
    "ddl_acc_f32": [I, P, P, L, P],
    # step glue (elementwise.hip): tanh backward, zero-padded 2-D copies, adds into gradient slots,
    # the gradient-arena zero fill, the embedding backward's id sort
    "ddl_tanh_bwd": [I, P, P, P, L, P],
    "ddl_copy2d": [I, P, L, L, L, P, L, L, L, P],
    "ddl_add_into": [I, P, P, L, P],
    "ddl_zero": [P, L, P],
    "ddl_rows_add_row": [I, P, P, P, L, L, P],
    "ddl_seq_prepend_add": [I, P, P, P, P, L, L, L, P],
    "ddl_sort_ids_ok": [L, L],
    "ddl_sort_ids": [P, L, P, P, P],
    "ddl_drain_acc": [I, P, P, L, P],
    "ddl_acc_grad": [I, P, P, L, I, I, P],
    "ddl_softmax_topk": [I, P, L, I, I, P, P, P, P],
    "ddl_gemm_conv_multi": [I, I, P, P, P, P, P, L, I, P, P],
    "ddl_conv3x3": [P, P, P, I, I, I, I, I, P, P, P, P, P, P, I, P],
    "ddl_conv3x3_wgrad": [P, P, P, I, I, I, I, I, P, L, I, I, I, P],
    "ddl_stem_wgrad": [P, P, P, I, I, I, I, I, I, I, P, L, I, I, I, P],
    "ddl_stem_fwd": [P, P, P, I, I, I, I, P, I, P],
    "ddl_s2d_input": [P, I, I, I, I, I, P, I, I, P],
    "ddl_s2d_weight": [P, I, I, I, I, P, I, I, P],
    "ddl_skinny_gemm": [P, P, P, L, I, I, P, P, P, P, P, P, I, P],
    "ddl_stream_gemm": [P, P, P, L, I, I, P, P, P, P, P, P, I, P],
    "ddl_stream_wgrad_ws": [I, I],
    "ddl_bn_bwd": [I, P, P, P, P, P, P, L, I, I, P, P, P, P, P, P, I, P],
    "ddl_ln_supported": [I],
    "ddl_ln_fwd": [I, P, P, L, P, P, P, P, P, L, I, F, U64, F, P],
    "ddl_ln_bwd_nblk": [L],
    "ddl_ln_bwd": [I, P, P, P, L, P, P, P, P, P, P, P, L, I, I, P, U64, F, P, P, P, P],
    # elementwise.hip
    "ddl_gelu_fwd": [I, P, P, L, P],
    "ddl_gelu_bwd": [I, P, P, P, L, P],
    "ddl_dropout": [I, P, P, L, U64, F, P],
    "ddl_colsum_nblk": [L],
    "ddl_colsum": [I, P, L, I, P, P, I, I, P],
    "ddl_softmax_ce": [I, P, P, L, I, P, P, P, P],
    "ddl_scale_by": [I, P, P, P, L, P],
    "ddl_maxpool_fwd": [I, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "ddl_maxpool_bwd": [I, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "ddl_avgpool_fwd": [I, P, P, I, I, I, P],
    "ddl_avgpool_bwd": [I, P, P, I, I, I, P],
    "ddl_embedding_fwd": [I, P, P, P, L, I, P],
    "ddl_embedding_bwd": [I, P, P, P, P, L, L, I, I, P],
    "ddl_embedding_bwd_sorted": [I, P, P, P, P, P, L, I, I, P],
    # optim.hip
    "ddl_sgd_step": [I, P, P, I, P, P, P, I, P, F, F, F, I, I, P],
    "ddl_adamw_step": [I, P, P, I, P, P, P, P, I, P, F, F, F, F, F, F, F, P],
    "ddl_lamb_step": [I, P, P, I, P, P, P, P, I, P, F, F, F, F, F, F, F, P, P],
    "ddl_sumsq": [I, P, L, P, P],
    "ddl_lamb_phase1": [I, P, P, P, P, P, I, P, F, F, F, F, F, F, P, P],
    "ddl_lamb_phase2": [P, I, P, P, P, P, I, F, F, F, F, F, P, P],
}
_fns = {}


def fn(name: str):
    """Typed handle to a C entry point (argtypes from _SIGS, int return)."""
    f = _fns.get(name)
    if f is None:
        f = getattr(get(), name)
        if name in _SIGS:
            f.argtypes = _SIGS[name]
        f.restype = ctypes.c_int
        _fns[name] = f
    return f


def call(name: str, *args) -> None:
    """Call a launcher on the current stream (stream appended automatically)."""
    rc = fn(name)(*args, stream())
    if rc != 0:
        raise RuntimeError(f"native kernel {name} failed with code {rc}")


def register(sigs: dict) -> None:
    _SIGS.update(sigs)


def dcode(t: torch.Tensor) -> int:
    """dtype code used by the C ABI: 0 fp32, 1 bf16."""
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError(f"native kernels support fp32/bf16, got {t.dtype}")


def p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


# ------------------------------------------------------------------ gradient sinks
# When a DataParallel reducer owns a parameter's gradient (a view into the flat
# gradient arena), the native backward kernels accumulate the weight gradient
# straight into that view in their epilogue and signal readiness to the reducer,
# instead of returning a tensor that autograd would add into the arena with an
# extra elementwise kernel per parameter.
def grad_sink(param) -> Optional[torch.Tensor]:
    if param is None:
        return None
    return getattr(param, "_ddl_main_grad", None)


def grad_ready(param) -> None:
    cb = getattr(param, "_ddl_grad_ready", None)
    if cb is not None:
        cb()


# ------------------------------------------------------------------ concurrent weight gradients
# A layer's input gradient (dgrad) and its weight gradient (wgrad) are independent GEMMs.
# With DDL_WGRAD_STREAM=1 the wgrad is issued on a side stream, ordered after everything
# the compute stream has issued so far (its operands, the arena's zeroing), and the compute
# stream joins it right after: the two GEMMs of ONE layer run concurrently -- a dgrad
# whose tile grid leaves CUs idle (BERT's N = 768 GEMMs: 192 tiles on 256 CUs) shares the
# chip with the wgrad -- while the next layer's backward and the gradient reducer's
# bucket launch (ordered after the compute stream) still see the finished gradient.
import contextlib as _contextlib  # noqa: E402

_WGRAD_STREAM = os.environ.get("DDL_WGRAD_STREAM", "0") != "0"
_side: dict = {}


def wgrad_stream_enabled() -> bool:
    return _WGRAD_STREAM


def set_wgrad_stream(enabled: bool) -> None:
    global _WGRAD_STREAM
    _WGRAD_STREAM = bool(enabled)


def fork_event():
    """The point of the compute stream a side-stream wgrad may start from: recorded BEFORE the
    layer's dgrad is launched (its operands -- the incoming gradient and the saved input --
    are ready there), so the two GEMMs run concurrently.  Ordered after the dgrad instead
    (``side_stream`` without ``after``), the side stream waited the dgrad out and the "overlap"
    was a serialisation plus two stream hops per layer.  None when the side stream is off."""
    if not _WGRAD_STREAM or not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
        return None
    ev = torch.cuda.Event()
    ev.record()
    return ev


@_contextlib.contextmanager
def side_stream(*tensors: torch.Tensor, after=None):
    """Run the block on this device's side stream (when enabled and not capturing), then
    make the compute stream wait for it.  ``after``: the ``fork_event`` the side stream starts
    from (default: everything the compute stream issued so far).  ``tensors`` are the block's
    inputs allocated on the compute stream: recorded on the side stream so the caching
    allocator does not hand their memory out again before the side stream is done with it."""
    if not _WGRAD_STREAM or not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
        yield
        return
    compute = torch.cuda.current_stream()
    dev = compute.device
    s = _side.get(dev)
    if s is None:
        s = _side[dev] = torch.cuda.Stream(device=dev)
    if after is not None:
        s.wait_event(after)
    else:
        s.wait_stream(compute)
    with torch.cuda.stream(s):
        yield
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(s)
    compute.wait_stream(s)
