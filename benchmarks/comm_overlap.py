#!/usr/bin/env python3
"""GEMM time with CUs taken by a concurrent collective (1 GPU stand-in).

An RCCL all-reduce overlapped with backward keeps one resident workgroup per
channel on its CUs for the whole collective.  A 256x256 GEMM block needs a whole
CU (256 VGPRs x 2 waves per SIMD, 128 KB LDS), so it cannot start on such a CU.
This script parks ``--occupy`` workgroups (``ddl_occupy``: one per CU, spinning on
the real-time counter) on a side stream and times back-to-back GEMMs of the
BERT-base / ResNet-50 shapes on the compute stream beside them, against the same
GEMMs alone.

    DDL_GEMM_DYNAMIC=0 python benchmarks/comm_overlap.py   # static tile striding
    DDL_GEMM_DYNAMIC=1 python benchmarks/comm_overlap.py   # per-XCD tile tickets

Prints one JSON line per (shape, occupancy).
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [  # name, mode, M, N, K, act
    ("bert_ffn1_gelu", 0, 16384, 3072, 768, "gelu"),
    ("bert_ffn1_gelu_noaux", 0, 16384, 3072, 768, "gelu_noaux"),   # GELU without the pre-activation store
    ("bert_ffn1_plain", 0, 16384, 3072, 768, None),
    ("bert_ffn2", 0, 16384, 768, 3072, None),
    ("bert_qkv", 0, 16384, 2304, 768, None),
    ("r50_1x1_64to256", 0, 802816, 256, 64, None),
    ("sq8192", 0, 8192, 8192, 8192, None),
    ("bert_nn_dgrad", 1, 16384, 768, 3072, None),       # dx = dy W (W reduction-outer)
    ("bert_nn_dgelu", 1, 16384, 3072, 768, "dgelu"),    # FFN1 dgrad * GELU'(z) + bias-grad sums
    ("bert_tn_wgrad_3072x768", 2, 3072, 768, 16384, None),   # dW = dy^T x (split-K)
    ("bert_tn_wgrad_768x3072", 2, 768, 3072, 16384, None),
]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--occupy", type=int, nargs="*", default=[0, 16, 32, 64])
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    from databricks_distributed_deep_learning_amd.ops import _lib
    from databricks_distributed_deep_learning_amd.ops._native_gemm import gemm
    lib = _lib.get()
    occ = lib.ddl_occupy
    occ.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
    occ.restype = ctypes.c_int
    dev = torch.device("cuda")
    sink = torch.zeros(256, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(priority=-1)
    dyn = os.environ.get("DDL_GEMM_DYNAMIC", "1")
    for name, mode, M, N, K, act in SHAPES:
        # operand layouts: NT A[M,K] B[N,K]; NN A[M,K] B[K,N]; TN A[K,M] B[K,N]
        a = torch.randn(*((K, M) if mode == 2 else (M, K)), device=dev).to(torch.bfloat16)
        w = torch.randn(*((N, K) if mode == 0 else (K, N)), device=dev).to(torch.bfloat16)
        lda = M if mode == 2 else K
        ldb = K if mode == 0 else N
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        bias = torch.randn(N, device=dev).to(torch.bfloat16) if act in ("gelu", "gelu_noaux") else None
        z = torch.empty_like(c) if act == "gelu" else None
        stats = None
        if act == "dgelu":
            z = torch.randn_like(c)
            stats = torch.empty((M + 127) // 128 * 2 * N, device=dev)
        act_k = "gelu" if act == "gelu_noaux" else act

        def run():
            gemm(mode, a, lda, w, ldb, c, N, M, N, K, bias=bias, act=act_k, aux=z, kernel="big",
                 colstats=stats)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        e1.synchronize()
        alone_ms = e0.elapsed_time(e1) / args.iters
        for nb in args.occupy:
            torch.cuda.synchronize()
            # the occupant outlives the timed GEMMs (3x their standalone time + 1 ms)
            usec = 1000.0 * (3 * alone_ms * args.iters) + 1000.0
            with torch.cuda.stream(side):
                rc = occ(nb, usec, sink.data_ptr(), ctypes.c_void_p(side.cuda_stream))
                assert rc == 0, rc
            torch.cuda._sleep(2_000_000)   # let the occupant's workgroups land first
            e0.record()
            for _ in range(args.iters):
                run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            torch.cuda.synchronize()
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "dynamic": dyn, "occupied_cus": nb,
                              "alone_ms": round(alone_ms, 4), "ms": round(ms, 4),
                              "slowdown": round(ms / alone_ms, 3),
                              "cu_share_left": round((256 - nb) / 256, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
