"""Memory trace of an auto-batched preset: the fitted batch (``utils/memory.py`` last_fit), then the peak
allocation of every warm-up step as ``Trainer._run`` runs them (online GEMM tuning on for transformers),
and the GEMM plan-table hits / misses -- to see what the real step allocates that the probe did not.

    python scripts/debug/autobatch_mem.py bert_large_lamb [--batch 0] [--steps 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from databricks_distributed_deep_learning_amd import get_preset  # noqa: E402
from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG  # noqa: E402
from databricks_distributed_deep_learning_amd.parallel import dist as ddist  # noqa: E402
from databricks_distributed_deep_learning_amd.training.loop import Trainer  # noqa: E402


def gb(x):
    return round(x / 2**30, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("preset")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    cfg = get_preset(a.preset)
    cfg.batch_size = a.batch
    tr = Trainer(cfg)
    dev = tr.device
    print("fit", tr.auto_batch, "batch", cfg.batch_size, "alloc", gb(torch.cuda.memory_allocated(dev)), flush=True)
    print("plan", NG.plan_stats(), flush=True)
    transformer = cfg.model.startswith(("bert", "vit"))
    with NG.online_tuning(enabled=True, default=transformer, max_mb=float("inf") if transformer else 0.0):
        for i in range(a.steps):
            torch.cuda.reset_peak_memory_stats(dev)
            try:
                tr.train_step()
                torch.cuda.synchronize(dev)
            except torch.cuda.OutOfMemoryError as e:
                print(f"step {i}: OOM ({str(e)[:160]}) peak {gb(torch.cuda.max_memory_allocated(dev))}", flush=True)
                raise
            NG.online_collect()
            print(f"step {i}: peak {gb(torch.cuda.max_memory_allocated(dev))} GB, alloc "
                  f"{gb(torch.cuda.memory_allocated(dev))} GB, plan {NG.plan_stats()}", flush=True)
    tr.close()
    ddist.destroy()




def compare(preset: str, b: int) -> None:
    """Peak of the fitter's probe vs the trainer's real step at one batch (both after a warm call)."""
    cfg = get_preset(preset)
    cfg.batch_size = b
    tr = Trainer(cfg)
    dev = tr.device

    def peak(fn):
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(dev)
        base = torch.cuda.memory_allocated(dev)
        fn()
        torch.cuda.synchronize(dev)
        return gb(torch.cuda.max_memory_allocated(dev) - base), gb(base)

    def probe():
        ld = tr._make_loader()
        tr.ddp.zero_grad()
        with tr.ddp.no_sync():
            loss = tr.loss_fn(ld.next())
            loss.backward()
        tr.ddp.zero_grad()

    def micro_nosync():
        tr.ddp.zero_grad()
        with tr.ddp.no_sync():
            loss = tr.loss_fn(tr.loader.next())
            loss.backward()

    for name, fn in [("probe", probe), ("probe", probe), ("micro_nosync", micro_nosync),
                     ("train_step", tr.train_step), ("train_step", tr.train_step), ("probe", probe)]:
        print(f"b={b} {name}: peak-over-base, base (GB) = {peak(fn)}", flush=True)
    tr.close()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "--compare":
        compare(sys.argv[1], int(sys.argv[3]))
        ddist.destroy()
    else:
        main()
