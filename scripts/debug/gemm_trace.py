"""Per-GEMM device time of one training step, grouped by call signature (GPU diagnostics).

    python scripts/debug/gemm_trace.py [resnet50|bert_base|vit_b16|bert_large] [--batch N]

Runs warm-up steps (GEMM tuning), then one traced step with HIP events around every
native GEMM launch, and prints the signatures sorted by time: which convolution /
Linear (forward, dgrad or wgrad), which kernel the tuner chose, and its TFLOP/s.
"""
import argparse
import collections
import sys

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd.config import get_preset  # noqa: E402
from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG  # noqa: E402
from databricks_distributed_deep_learning_amd.training.loop import Trainer  # noqa: E402

MODES = {0: "NT", 1: "NN", 2: "TN", 3: "CONV", 4: "CONVW", 5: "CONVW_A"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="resnet50")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    if a.model == "vit_b16":
        cfg = get_preset("vit_b16", **({"batch_size": a.batch} if a.batch else {}))
    elif a.model == "bert_large":
        cfg = get_preset("bert_large_lamb", batch_size=a.batch or 32, grad_accum=1)
    else:
        preset = "resnet50_ddp" if a.model.startswith("resnet") else "bert_base_ddp"
        cfg = get_preset(preset, batch_size=a.batch or (256 if preset.startswith("resnet") else 128))
        cfg = cfg.replace(model=a.model)
    cfg = cfg.replace(steps=1, warmup_steps=2, log_every=0)
    tr = Trainer(cfg)
    tr.run()                       # warm-up + tuning
    torch.cuda.synchronize()
    NG.trace(True)
    tr.train_step()
    torch.cuda.synchronize()
    recs = NG.trace(False)
    agg = collections.defaultdict(lambda: [0.0, 0, None])
    for sig, choice, e0, e1 in recs:
        k = (sig, choice)
        agg[k][0] += e0.elapsed_time(e1)
        agg[k][1] += 1
    total = sum(v[0] for v in agg.values())
    print(f"{len(recs)} GEMM launches, {total:.2f} ms of GEMM time in one step")
    print("| mode | M | N | K | conv (N,H,W,C,P,Q,s,...) | epilogue | kernel | calls | ms | TF/s |")
    print("|---|---:|---:|---:|---|---|---|---:|---:|---:|")
    for (sig, choice), (ms, n, _) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        mode, M, N, K, conv, act, bias, res, stats, acc = sig
        epi = ",".join(t for t, on in (("bias", bias), (str(act), act), ("res", res), ("stats", stats),
                                       ("acc", acc)) if on)
        cv = "" if conv is None else str(conv[:7])
        tf = 2.0 * M * N * K * n / (ms * 1e9)
        print(f"| {MODES.get(mode & 15, mode)}{'^T' if mode & 16 else ''} | {M} | {N} | {K} | {cv} | {epi} | "
              f"{choice[0]}x{choice[1]} | {n} | {ms:.3f} | {tf:.0f} |")


if __name__ == "__main__":
    main()
