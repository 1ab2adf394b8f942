#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 images/sec (+ BERT-base samples/sec), whole node.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it
is launched by ``torch.distributed.run`` (one rank per GPU, RCCL over xGMI).
W untimed warm-up steps, then EXACTLY K optimizer steps timed between
barrier + device synchronisation on both sides; the max over ranks is the step
time.  Rank 0 prints ONE JSON line on stdout (everything else goes to stderr).

``python bench.py --gpus N`` with N > 1 and no launcher environment (no
``WORLD_SIZE``) launches the N ranks itself: N child processes of this script with
the torchrun variables set, started BEFORE anything in the parent touches the GPU
(the parent never imports torch); the parent relays rank 0's JSON line and exits
with the first failing child's code (the others are terminated).

``--native stock`` measures the stock PyTorch-ROCm arm instead: plain nn.Conv2d /
nn.BatchNorm2d / nn.Linear / SDPA models under bf16 autocast with fused torch
optimizers and torch DistributedDataParallel (``baselines/stock.py``).

Workload (BASELINE.json:8,9): ResNet-50 bf16 data-parallel training on synthetic
ImageNet-shape batches (NHWC 224x224, 1000 classes, SGD-momentum, fp32 master
weights), random-init weights; weak scaling (fixed per-GPU batch).  BERT-base
seq-128 fine-tuning (AdamW) is measured in the same run and reported under
``extra`` (``--model resnet50`` skips it).

A/B switches read from the environment: ``DDL_PHASE_TIMING=0`` (no per-phase events),
``DDL_EAGER_OPTIMIZER=1`` (per-bucket optimizer updates during backward on a side stream;
measured slower on one GPU, ``profiles/ab_r03.md``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def self_launch(n: int) -> int:
    """Run this script as ``n`` local ranks (one per GPU) and relay rank 0's stdout."""
    import socket
    import subprocess
    import tempfile
    import time
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log(f"[bench] rank {procs.index(p)} exited with {code}; stopping the others")
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    out.seek(0)
    sys.stdout.write(out.read())
    sys.stdout.flush()
    return rc


# per-GPU micro-batch defaults of the extra configs (BASELINE.json:10-11); BERT-large: seq 512,
# LAMB, 4 micro-batches per optimizer step (the train CLI's preset sizes its batch to HBM instead)
_EXTRA = {"vit_b16": dict(preset="vit_b16", batch=128, seq=None, accum=1),
          "bert_large": dict(preset="bert_large_lamb", batch=32, seq=512, accum=4)}


def run_one(model: str, args, world: int):
    if args.native == "stock":
        from databricks_distributed_deep_learning_amd.baselines import run_stock
        if model in _EXTRA:
            e = _EXTRA[model]
            return run_stock(model, args.batch or e["batch"], args.steps, args.warmup, seq_len=e["seq"] or 128,
                             bucket_mb=args.bucket_mb or 25.0, grad_accum=e["accum"],
                             dropout=0.0 if model == "vit_b16" else 0.1)
        batch = (args.batch or 256) if model == "resnet50" else (args.bert_batch or 128)
        return run_stock(model, batch, args.steps, args.warmup, seq_len=128, bucket_mb=args.bucket_mb or 25.0,
                         pad_fraction=args.bert_pad_fraction)
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    if model == "resnet50":
        cfg = get_preset("resnet50_ddp", batch_size=args.batch or 256)
    elif model in _EXTRA:
        e = _EXTRA[model]
        cfg = get_preset(e["preset"], batch_size=args.batch or e["batch"])
    else:
        # --bert-pad-fraction > 0: HF-style right-padded batches with an attention mask (the
        # masked attention path a real fine-tune runs); 0 = full-length sequences, no mask
        cfg = get_preset("bert_base_ddp", batch_size=args.bert_batch or 128, dropout=0.1,
                         pad_fraction=args.bert_pad_fraction)
    cfg = cfg.replace(steps=args.steps, warmup_steps=args.warmup, native=args.native, log_every=0,
                      bucket_mb=args.bucket_mb, backend=args.backend,
                      zero_optimizer=args.zero, sync_bn=args.sync_bn, dp_rehearsal=args.dp_rehearsal,
                      eager_optimizer=os.environ.get("DDL_EAGER_OPTIMIZER", "0") == "1",
                      phase_timing=os.environ.get("DDL_PHASE_TIMING", "1") != "0")
    from databricks_distributed_deep_learning_amd.ops import _native_gemm
    with _native_gemm.plan_usage() as used:
        tr = Trainer(cfg)
        s = tr.run()
        tr.close()
        del tr
    s["gemm_plan"] = gemm_plan_digest(model, used)
    s["plan_source"] = _native_gemm.plan_stats()
    return s


def gemm_plan_digest(model: str, used) -> str:
    """Hash of the GEMM kernel plan this model ran: every signature it looked up -> (kernel,
    splits), whether from the committed plan table or tuned in this process; the full plan goes to
    stderr.  Two bench processes whose step times differ can then be told apart by plan or not
    (same plan: the cause is elsewhere)."""
    import hashlib
    from databricks_distributed_deep_learning_amd.ops import _native_gemm
    plan = {k: list(v) for k, v in sorted(_native_gemm.current_plan(used).items())}
    if not plan:
        return ""
    text = json.dumps(plan, sort_keys=True)
    digest = hashlib.sha1(text.encode()).hexdigest()[:12]
    log(f"[bench] {model} gemm plan {digest} ({len(plan)} signatures): {text}")
    tim = {k: {f"{c[0]}:{c[1]}": round(t * 1000.0, 1) for c, t in v.items()}
           for k, v in sorted(_native_gemm._timings.items()) if k in plan}
    log(f"[bench] {model} gemm candidate us ({_native_gemm.online_stats()}): {json.dumps(tim)}")
    return digest


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="both", choices=["both", "resnet50", "bert_base", "vit_b16", "bert_large"],
                    help="both = the headline pair; vit_b16 / bert_large: the other BASELINE configs")
    ap.add_argument("--batch", type=int, default=0, help="ResNet-50 per-GPU batch (default 256)")
    ap.add_argument("--bert-batch", type=int, default=0, help="BERT-base per-GPU batch (default 128)")
    ap.add_argument("--bert-pad-fraction", type=float, default=0.0,
                    help="BERT: random right-padding up to this fraction of the sequence, with attention mask")
    ap.add_argument("--native", default="auto", choices=["auto", "on", "off", "stock"],
                    help="auto/on: HIP kernels; stock: plain PyTorch-ROCm + torch DDP arm; "
                         "off: the framework's CPU-oracle ops (correctness reference, not a baseline)")
    ap.add_argument("--bucket-mb", default="auto",
                    help="gradient bucket MB, or 'auto' (default: sized from the startup all-reduce probe at "
                         "N > 1; 4 / 25 MB without a probe -- bucket_policy.source in the output says which)")
    ap.add_argument("--dp-rehearsal", action="store_true",
                    help="N = 1: run the N > 1 step form anyway (native RCCL engine, per-bucket all-reduces, "
                         "per-bucket range optimizer) so its cost shows in phases_ms")
    ap.add_argument("--zero", action="store_true", help="ZeRO-1: shard fp32 master + optimizer state over ranks")
    ap.add_argument("--sync-bn", action="store_true", help="SyncBatchNorm (CV models)")
    ap.add_argument("--backend", default=os.environ.get("DDL_BACKEND", "auto"),
                    help="process-group backend (auto = RCCL on GPU); gloo only for 1-GPU multi-rank rehearsals")
    args = ap.parse_args()
    args.bucket_mb = 0.0 if str(args.bucket_mb).lower() == "auto" else float(args.bucket_mb)
    # the first step times GEMM kernel candidates per shape (ops/_native_gemm.py);
    # it must never land inside the timed region
    args.warmup = max(1, args.warmup)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args.gpus)

    import torch
    from databricks_distributed_deep_learning_amd.parallel import dist as ddist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    ddist.init(args.backend)
    world = ddist.world_size()
    results = {}
    order = ["resnet50", "bert_base"] if args.model == "both" else [args.model]
    for m in order:
        results[m] = run_one(m, args, world)
        log(f"[bench] {m}: {json.dumps(results[m])}")
        torch.cuda.empty_cache() if torch.cuda.is_available() else None

    head = results.get("resnet50") or results[order[0]]
    is_r50 = "resnet50" in results
    names = {"resnet50": "ResNet-50 images/sec", "bert_base": "BERT-base samples/sec",
             "vit_b16": "ViT-B/16 images/sec", "bert_large": "BERT-large (seq 512, LAMB) samples/sec"}
    line = {
        "metric": names[order[0] if not is_r50 else "resnet50"] + " (whole node)",
        "value": round(head["samples_per_sec"], 2),
        "unit": "images/s" if (is_r50 or order[0] == "vit_b16") else "samples/s",
        "n_gpus": ddist.world_size(),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(head["ms_per_step"], 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,   # BASELINE.json "published": {} — the reference publishes no number
        "dtype": "bf16",
        "data": "synthetic (device-resident random NHWC images / token ids), random-init weights",
        "config": {
            "model": head["model"],
            "global_batch": head["global_batch"],
            "per_gpu_batch": head["per_rank_batch"],
            "seq_len": head["seq_len"],
            "image_size": 224 if head.get("task") == "cv" else None,
            "grad_accum": head.get("grad_accum", 1),
            "optimizer": head["optimizer"],
            "parallelism": f"dp{ddist.world_size()}",
            "native_kernels": head["native"],
            "grad_comm": head.get("comm"),
        },
        "phases_ms": head.get("phases_ms"),
        "gemm_plan": {m: r.get("gemm_plan", "") for m, r in results.items()},
        # committed plan table (ops/gemm_plans.json) vs tuned: source, table hits, misses (tuned here)
        "plan_source": {k: v for k, v in (head.get("plan_source") or {}).items()
                        if k in ("source", "table_hits", "misses", "status", "gemm_src_hash")},
        "bucket_policy": head.get("bucket_policy"),
    }
    if head.get("comm_probe"):
        line["comm_probe"] = head["comm_probe"]          # startup all-reduce probe (N > 1, native engine)
    if head.get("comm_buckets"):
        line["comm_buckets"] = head["comm_buckets"]      # last step: per-bucket ring time / bus GB/s
    for k in ("rccl", "rank_devices", "dp_rehearsal"):    # RCCL's nranks / device; every rank's device
        if head.get(k):
            line[k] = head[k]
    if "bert_base" in results and is_r50:
        b = results["bert_base"]
        line["extra"] = {
            "bert_base_samples_per_sec": round(b["samples_per_sec"], 2),
            "bert_base_ms_per_step": round(b["ms_per_step"], 3),
            "bert_base_global_batch": b["global_batch"],
            "bert_base_seq_len": b["seq_len"],
        }
    if ddist.is_main():
        print(json.dumps(line), flush=True)
    ddist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
