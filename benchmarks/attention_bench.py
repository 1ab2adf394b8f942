#!/usr/bin/env python3
"""Fused attention (K14/K15) timing on the BERT-base / BERT-large / ViT-B shapes.

    python benchmarks/attention_bench.py [--shapes bert_base,vit,bert_large]

Per shape: forward and forward+backward wall time (HIP events, median of 5 x 20
calls), with / without probability dropout and with / without a key-padding mask,
and the achieved TFLOP/s (4*B*H*S^2*64 forward, 2.5x that for the backward).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = {"bert_base": (128, 128, 12), "vit": (128, 197, 12), "bert_large": (16, 512, 16)}


def timeit(fn, iters=20, reps=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) / iters)
    return statistics.median(out)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="bert_base,vit,bert_large")
    args = ap.parse_args()
    from databricks_distributed_deep_learning_amd.ops import _native_attention as NA
    dev = torch.device("cuda")
    for name in args.shapes.split(","):
        B, S, H = SHAPES[name]
        qkv = torch.randn(B, S, 3 * H * 64, device=dev).to(torch.bfloat16).requires_grad_(True)
        g = torch.randn(B, S, H * 64, device=dev).to(torch.bfloat16)
        zmask = torch.zeros(B, S, device=dev)
        fl = 4.0 * B * H * S * S * 64
        for p in (0.0, 0.1):
            for mask in (None, zmask):
                def fwd():
                    with torch.no_grad():
                        NA.attention(qkv, H, mask, p)

                def fwdbwd():
                    out = NA.attention(qkv, H, mask, p)
                    out.backward(g)
                tf = timeit(fwd)
                tfb = timeit(fwdbwd)
                print(json.dumps({"shape": name, "B": B, "S": S, "H": H, "p_drop": p, "mask": mask is not None,
                                  "fwd_ms": round(tf, 4), "bwd_ms": round(tfb - tf, 4),
                                  "fwd_tflops": round(fl / tf / 1e9, 1),
                                  "bwd_tflops": round(2.5 * fl / max(1e-6, tfb - tf) / 1e9, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
