"""Notebook-style ``train(cfg)`` for CV and NLP (north-star N4).

The same function runs in a notebook cell (world 1, no launcher), under
``Distributor(8).run(train, cfg)`` / ``HorovodRunner(8).run(train, cfg=cfg)``,
and under ``torchrun``.  Per rank:

    model (random init, bf16 params) -> flat ParamArena -> DataParallel reducer
    -> flat optimizer (fp32 master) -> synthetic device-resident loader
    for step: [micro-steps under no_sync] fwd, bwd (bucketed RCCL all-reduce
              overlapped with backward) -> finish() -> fused optimizer step

Returns a summary dict (rank-aggregated throughput, final loss, config).
"""
from __future__ import annotations

import contextlib
import math
import os
import sys
import time
from typing import Any, Callable, Dict, Optional

import torch

from .. import ops
from ..config import TrainConfig, apply_overrides
from ..data import SyntheticImageNet, SyntheticTokens
from ..models import build_model, cast_params, convert_sync_batchnorm, count_params
from ..optim import LRSchedule, ParamArena, build_optimizer
from ..parallel import dist as ddist
from ..parallel.ddp import DataParallel
from ..utils import checkpoint as ckpt
from ..utils import profiling
from ..utils.faults import maybe_fail
from ..utils.metrics import JsonlLogger, PhaseTimer, StepTimer, ThroughputMeter, memory_stats

DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}


class Trainer:
    """Holds the per-rank training state; ``train()`` is the notebook-facing wrapper."""

    def __init__(self, cfg: TrainConfig):
        self.cfg = cfg
        ddist.init(cfg.backend)
        self.device = ddist.device()
        if cfg.native != "auto":
            ops.set_native_mode("off" if cfg.native == "off" else "auto")
        self.rank, self.world = ddist.rank(), ddist.world_size()
        self.dtype = DTYPES[cfg.dtype]
        self.task = cfg.resolved_task
        torch.manual_seed(cfg.seed)
        model = build_model(cfg.model, num_classes=cfg.num_classes, dropout=cfg.dropout,
                            image_size=cfg.image_size)
        model = model.to(self.device)
        cast_params(model, self.dtype)
        if cfg.sync_bn and self.world > 1:
            convert_sync_batchnorm(model)
        self.model = model
        self.n_params = count_params(model)
        zero = cfg.zero_optimizer and self.world > 1
        self.arena = ParamArena(list(model.named_parameters()), pad_multiple=self.world * 64 if zero else 1)
        accumulate_fp32 = cfg.grad_accum > 1 and self.dtype != torch.float32
        rd = {"auto": None, "fp32": torch.float32, "bf16": torch.bfloat16}[cfg.grad_reduce_dtype]
        comm, self.comm_probe = self._comm_engine(rd)
        bucket_mb, first_mb = cfg.bucket_mb, cfg.first_bucket_mb
        if bucket_mb <= 0:      # "auto": sized from the probe (fixed defaults without one)
            from ..parallel.comm import auto_buckets
            esz = torch.empty((), dtype=rd or self.arena.dtype).element_size()
            first_mb, bucket_mb = auto_buckets(self.comm_probe, self.arena.numel * esz / 2 ** 20) \
                if self.comm_probe else (4.0, 25.0)
        self.bucket_policy = {"bucket_mb": bucket_mb, "first_bucket_mb": first_mb,
                              "source": ("probe" if self.comm_probe else "default") if cfg.bucket_mb <= 0
                              else "config"}
        # LAMB's trust ratio needs every tensor whole in one optimizer range: no split tensors
        self.ddp = DataParallel(model, self.arena, bucket_mb=bucket_mb, first_bucket_mb=first_mb,
                                reduce_dtype=rd, broadcast_buffers=cfg.broadcast_buffers,
                                accumulate_fp32=accumulate_fp32, comm=comm, shard=zero,
                                split_tensors=cfg.resolved_optimizer != "lamb")
        # ZeRO-1: the optimizer owns chunk `rank` of every reduce-scattered bucket and hands its
        # updated chunks back through the reducer's overlapped per-bucket all-gathers
        self.opt = build_optimizer(cfg.resolved_optimizer, self.arena, cfg,
                                   shard=(self.rank, self.world, self.ddp.shard_groups()) if zero else None)
        if zero:
            self.opt.gather_fn = self.ddp.gather_params
        self.sched = LRSchedule(cfg.lr, cfg.lr_schedule, cfg.lr_warmup_steps, cfg.steps + cfg.warmup_steps)
        self.overlap_optimizer = ((self.world > 1 or self.rehearsal) and cfg.overlap_optimizer
                                  and self.opt.supports_ranges() and self.ddp.reduce_dtype == self.arena.dtype)
        # on the GPU the per-bucket updates start DURING backward, on a side stream, as soon as a
        # bucket's gradients (and its all-reduce) are done (DataParallel.set_eager)
        self.eager_optimizer = (cfg.overlap_optimizer and cfg.eager_optimizer and self.opt.supports_ranges()
                                and os.environ.get("DDL_EAGER_OPTIMIZER", "1") != "0"
                                and self.ddp.reduce_dtype == self.arena.dtype and self.arena.grad.is_cuda)
        self.auto_batch = None
        if cfg.batch_size <= 0:
            cfg.batch_size = self._auto_batch()
            from ..utils.memory import last_fit
            self.auto_batch = dict(last_fit)
            if ddist.is_main():
                print(f"[auto-batch] per-rank batch {cfg.batch_size}: {self.auto_batch}", file=sys.stderr, flush=True)
        self.loader = self._make_loader()
        self.step = 0
        self.logger = JsonlLogger(cfg.log_file, enabled=ddist.is_main())
        self.phases = PhaseTimer(self.device, enabled=cfg.phase_timing)
        if cfg.resume and cfg.checkpoint_dir and ckpt.latest(cfg.checkpoint_dir):
            meta = ckpt.load(cfg.checkpoint_dir, model, self.opt, loader=self.loader)
            self.step = int(meta["step"])

    # ------------------------------------------------------------------
    def _comm_engine(self, reduce_dtype):
        """(comm argument for DataParallel, probe results).  With several ranks on GPUs and
        the native engine available, the engine is created here so it can be probed
        (``parallel.comm.probe_allreduce``: 1 / 4 / 16 / 64 MB all-reduces, bus GB/s) before
        the buckets are laid out -- ``bucket_mb <= 0`` sizes them from the probe."""
        c = self.cfg
        # (the watchdog runs from the engine's construction on, so a peer lost during the probe
        # aborts the communicator instead of hanging the rank)
        self.rehearsal = False
        from ..parallel.comm import CommError, NativeComm, TorchCollectives, native_available, probe_allreduce

        def torch_path(comm):
            # no native engine: the auto bucket policy still probes, over the process group itself
            # (gloo on the CPU: smaller messages, the same latency-bandwidth fit)
            if self.world > 1 and (c.comm_probe or c.bucket_mb <= 0):
                cpu = self.device.type != "cuda"
                sizes = (0.25, 1, 4) if cpu else (1, 4, 16, 64)
                return comm, probe_allreduce(TorchCollectives(), self.device, sizes_mb=sizes, iters=3 if cpu else 5,
                                             dtype=reduce_dtype or self.arena.dtype, world=self.world)
            return comm, []
        if c.comm not in ("auto", "native") or self.device.type != "cuda":
            return torch_path(c.comm)
        if self.world == 1 and not c.dp_rehearsal:
            return c.comm, []
        if not native_available():
            return torch_path(c.comm)
        try:
            eng = NativeComm()
        except CommError:
            if c.comm == "native":
                raise
            return torch_path("torch")
        self.rehearsal = self.world == 1
        probe = []
        if self.world > 1 and (c.comm_probe or c.bucket_mb <= 0):
            probe = probe_allreduce(eng, self.device, dtype=reduce_dtype or self.arena.dtype, world=self.world)
        return eng, probe

    def _make_loader(self):
        c = self.cfg
        if self.task == "cv":
            return SyntheticImageNet(c.batch_size, c.image_size, c.num_classes, self.device, self.dtype,
                                     rank=self.rank, seed=c.seed, pool=c.synthetic_pool)
        mc = getattr(self.model, "config", None)
        vocab = min(c.vocab_size, getattr(mc, "vocab_size", c.vocab_size))
        return SyntheticTokens(c.batch_size, c.seq_len, vocab, c.num_classes, self.device,
                               rank=self.rank, seed=c.seed, pool=c.synthetic_pool, pad_fraction=c.pad_fraction)

    def _auto_batch(self) -> int:
        from ..utils.memory import fit_batch_size
        c = self.cfg

        def probe(b):
            old = c.batch_size
            c.batch_size = b
            ld = self._make_loader()
            self.ddp.zero_grad()
            with self.ddp.no_sync():
                loss = self.loss_fn(ld.next())
                loss.backward()
            self.ddp.zero_grad()
            c.batch_size = old
        return fit_batch_size(probe, self.device, start=8)

    def loss_fn(self, batch) -> torch.Tensor:
        if self.task == "cv":
            x, y = batch
            return ops.cross_entropy(self.model(x), y)
        loss, _ = self.model(batch["input_ids"], batch.get("attention_mask"), None, batch["labels"])
        return loss

    def train_step(self) -> torch.Tensor:
        """One optimizer step: grad_accum micro-steps (communication on the last), then
        the fused optimizer.  Phases are bracketed by roctx ranges (``DDL_ROCTX=1``, seen
        by ``rocprofv3 --marker-trace``) and HIP-event marks (:class:`PhaseTimer`)."""
        c = self.cfg
        ph = self.phases
        ph.begin()
        self.ddp.zero_grad()
        loss_sum = None
        scale = 1.0 / (self.world * c.grad_accum)
        for micro in range(c.grad_accum):
            batch = self.loader.next()
            last = micro == c.grad_accum - 1
            ctx = self.ddp.no_sync() if not last else contextlib.nullcontext()
            if last and self.eager_optimizer:
                self.opt.begin_step(lr=self.sched(self.step))
                self.ddp.set_eager(lambda g, lo, hi: self.opt.step_range(g, scale, lo, hi))
            with ctx:
                with profiling.range("fwd"):
                    loss = self.loss_fn(batch)
                ph.mark("fwd")
                with profiling.range("bwd"):
                    loss.backward(self._seed_grad(loss))
                ph.mark("bwd")
            loss_sum = loss.detach() if loss_sum is None else loss_sum + loss.detach()
            # drop this micro-step's graph now: the native autograd Functions keep operands on ctx
            # attributes, which live as long as the graph does -- held through the NEXT micro-step's
            # forward they cost BERT-large (batch 128 x seq 512) 11.4 GB over the fitter's one-micro-step
            # probe, and the fitted batch went out of memory (scripts/debug/autobatch_mem.py --compare)
            del loss
        if self.eager_optimizer:
            with profiling.range("comm_wait+opt"):
                self.ddp.finish()               # joins the side stream (or runs the remaining updates)
                self.ddp.set_eager(None)
                self.opt.end_step()
            ph.mark("comm_wait+opt")
        elif self.overlap_optimizer:
            # each bucket's optimizer update starts as soon as ITS all-reduce is done, so
            # the last buckets' rings (BERT's 68 MB embedding bucket) run under the update
            # of everything else instead of in front of it
            with profiling.range("comm_wait+opt"):
                self.opt.begin_step(lr=self.sched(self.step))
                self.ddp.finish(on_ready=lambda g, lo, hi: self.opt.step_range(g, scale, lo, hi))
                self.opt.end_step()
            ph.mark("comm_wait+opt")
        else:
            with profiling.range("comm_wait"):
                grad = self.ddp.finish()
            ph.mark("comm_wait")
            with profiling.range("opt"):
                self.opt.step(grad, grad_scale=scale, lr=self.sched(self.step))
            ph.mark("opt")
        ph.end_step()
        self.step += 1
        return loss_sum / c.grad_accum if c.grad_accum > 1 else loss_sum

    def _seed_grad(self, loss: torch.Tensor) -> torch.Tensor:
        """d(loss)/d(loss) = 1, one cached device scalar (``backward()`` would fill a new one per step)."""
        key = (loss.dtype, loss.device)
        g = self.__dict__.setdefault("_seed_grads", {}).get(key)
        if g is None:
            g = self._seed_grads[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
        return g

    def agree_kernel_plans(self, max_rounds: int = 3) -> None:
        """Data-parallel ranks run identical GEMM kernel plans (ops/_native_gemm.py
        ``agree_across_ranks``): a rank that tuned differently would gate every step.
        A changed plan can route GEMMs through signatures not tuned yet, so one more
        untimed step runs and the agreement repeats (same count on every rank: every
        rank computes the same answer)."""
        if self.world == 1 or not self.arena.flat.is_cuda:
            return
        from ..ops import _native_gemm
        for _ in range(max_rounds):
            if _native_gemm.agree_across_ranks() == 0:
                return
            self.train_step()

    def close(self) -> None:
        """Release the reducer's hooks and native communicator (the next Trainer in this
        process -- bench.py runs two -- then starts from a clean active-engine slot)."""
        self.ddp.close()

    def _abort_comm(self) -> None:
        """Failure path: abort the native RCCL communicator so collectives blocked on a
        dead peer return and this rank exits instead of hanging until the timeout."""
        eng = getattr(self.ddp, "native", None)
        if eng is not None and hasattr(eng, "close"):
            try:
                eng.close(abort=True)
            except Exception:  # noqa: BLE001 - already failing; keep the original error
                pass

    @property
    def samples_per_step(self) -> int:
        return self.cfg.batch_size * self.cfg.grad_accum * self.world

    def run(self, steps: Optional[int] = None, warmup: Optional[int] = None,
            callback: Optional[Callable[[int, float], None]] = None) -> Dict[str, Any]:
        try:
            return self._run(steps, warmup, callback)
        except BaseException:
            self._abort_comm()
            raise

    def _global_loss(self, loss: torch.Tensor) -> float:
        """Mean loss over ranks (collective C4; log points only)."""
        v = float(loss)
        if self.world > 1:
            v = ddist.all_reduce_scalars([v], op="sum")[0] / self.world
        return v

    def _run(self, steps, warmup, callback) -> Dict[str, Any]:
        c = self.cfg
        steps = c.steps if steps is None else steps
        warmup = c.warmup_steps if warmup is None else warmup
        self.model.train()
        # untuned GEMM signatures of transformer models pick their kernels from their own calls in
        # these warm-up steps (ops/_native_gemm.py online_tuning; DDL_GEMM_TUNE_ONLINE=0/1 overrides)
        from ..ops import _native_gemm
        transformer = c.model.startswith(("bert", "vit", "gpt", "t5", "roberta"))
        online_mb = float(os.environ.get("DDL_GEMM_ONLINE_MAX_MB", "inf" if transformer else "0"))
        with _native_gemm.online_tuning(enabled=self.device.type == "cuda", default=online_mb > 0,
                                        max_mb=online_mb):
            for _ in range(warmup):
                self.train_step()
                _native_gemm.online_collect()
        if warmup:
            self.agree_kernel_plans()
        _native_gemm.release_tuning_buffers()     # the tuner's 640 MB flush buffer back to the allocator
        self.phases.summary(reset=True)          # warm-up (and tuning) steps are not reported
        timer = StepTimer(self.device)
        meter = ThroughputMeter(self.samples_per_step)
        ddist.barrier()
        timer.start()
        t_seg = 0.0
        last = None
        for i in range(steps):
            maybe_fail(self.step, c.fault_rank, c.fault_step)
            loss = self.train_step()
            last = loss
            if c.log_every and (i + 1) % c.log_every == 0 and i != steps - 1:
                t_pause = timer.stop()            # log points are outside the timed region
                t_seg += t_pause
                gl = self._global_loss(loss)
                if callback:
                    callback(self.step, gl)
                self.logger.log({"step": self.step, "loss": gl, "lr": self.opt.lr,
                                 **self.phases.summary(reset=True), **memory_stats(self.device)})
                timer.start()
            if c.check_replicas_every and self.step % c.check_replicas_every == 0:
                t_seg += timer.stop()             # (outside the timed region, like log points)
                self.ddp.check_replicas()
                timer.start()
            if c.checkpoint_every and c.checkpoint_dir and self.step % c.checkpoint_every == 0:
                t_pause = timer.stop()
                t_seg += t_pause
                self.save_checkpoint()
                timer.start()
        self.ddp.wait_params()               # ZeRO-1: the last step's parameter all-gathers
        ddist.barrier()
        t_seg += timer.stop()
        meter.update(t_seg, steps)
        t_max = ddist.all_reduce_scalars([t_seg], op="max")[0]
        last_loss = self._global_loss(last) if last is not None else float("nan")
        phases = self.phases.summary(reset=True)
        if last is not None:
            if callback:
                callback(self.step, last_loss)
            self.logger.log({"step": self.step, "loss": last_loss, "lr": self.opt.lr, **phases,
                             **memory_stats(self.device)})
        summary = {
            "model": c.model, "task": self.task, "world_size": self.world, "steps": steps, "warmup": warmup,
            "per_rank_batch": c.batch_size, "grad_accum": c.grad_accum, "global_batch": self.samples_per_step,
            "seq_len": c.seq_len if self.task == "nlp" else None, "dtype": c.dtype,
            "optimizer": c.resolved_optimizer, "params": self.n_params,
            "seconds": t_max, "ms_per_step": 1000.0 * t_max / max(1, steps),
            "samples_per_sec": self.samples_per_step * steps / t_max if t_max > 0 else 0.0,
            "final_loss": last_loss, "native": ops.native_mode(),
            "buckets_mb": [round(b, 2) for b in self.ddp.bucket_sizes_mb()],
            "comm": self.ddp.comm, "phases_ms": {k: round(v, 3) for k, v in phases.items()},
            "bucket_policy": self.bucket_policy,
        }
        if self.auto_batch:
            summary["auto_batch"] = self.auto_batch
        if self.comm_probe:
            summary["comm_probe"] = self.comm_probe
        if self.rehearsal:
            summary["dp_rehearsal"] = True
        eng = getattr(self.ddp, "native", None)
        if eng is not None and hasattr(eng, "world"):
            # the communicator's own view of the job (what RCCL was initialised with)
            summary["rccl"] = {"nranks": int(eng.world), "rank": int(eng.rank), "device": int(eng.device.index),
                               "version": ".".join(str(v) for v in torch.cuda.nccl.version())}
        if self.world > 1 and self.device.type == "cuda":
            import socket
            summary["rank_devices"] = ddist.all_gather_object(
                {"rank": self.rank, "device": self.device.index, "host": socket.gethostname(),
                 "pci": torch.cuda.get_device_properties(self.device).pci_bus_id
                 if hasattr(torch.cuda.get_device_properties(self.device), "pci_bus_id") else None})
        timings = self.ddp.bucket_timings()       # the last step's rings (synchronised by the barrier above)
        if timings:
            summary["comm_buckets"] = timings
        summary.update(memory_stats(self.device))
        if c.checkpoint_dir and not c.checkpoint_every:
            self.save_checkpoint()
        return summary

    def save_checkpoint(self) -> None:
        self.ddp.wait_params()
        ckpt.save(self.cfg.checkpoint_dir, self.model, self.opt, self.step, self.cfg.to_dict(), loader=self.loader)


def train(cfg: Optional[TrainConfig] = None, **overrides) -> Dict[str, Any]:
    """Notebook-style entry point.  ``train(get_preset("resnet50_ddp"), steps=20)``."""
    cfg = (cfg or TrainConfig()).replace(**overrides) if overrides else (cfg or TrainConfig())
    trainer = Trainer(cfg)
    out = trainer.run()
    trainer.close()
    return out


def main(argv=None) -> int:
    """CLI: ``python -m databricks_distributed_deep_learning_amd.training.loop --preset resnet50_ddp --steps 20``."""
    import json
    import sys
    from ..config import get_preset
    argv = list(sys.argv[1:] if argv is None else argv)
    preset = "resnet50_ddp"
    if "--preset" in argv:
        i = argv.index("--preset")
        preset = argv[i + 1]
        del argv[i:i + 2]
    cfg = apply_overrides(get_preset(preset), argv)
    out = train(cfg)
    if ddist.is_main():
        print(json.dumps(out))
    ddist.destroy()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
