"""Distributed plumbing on CPU / gloo, world_size 2 (BASELINE.json:7)."""
import os

import pytest
import torch

from databricks_distributed_deep_learning_amd.parallel import ChildFailed, Distributor, HorovodRunner


# ---------------------------------------------------------------- helpers run in children
def _rank_info(tag):
    import torch.distributed as dist
    t = torch.tensor([dist.get_rank() + 1.0])
    dist.all_reduce(t)
    return {"tag": tag, "rank": dist.get_rank(), "world": dist.get_world_size(), "sum": t.item()}


def _fail_on_rank1():
    import torch.distributed as dist
    if dist.get_rank() == 1:
        raise ValueError("boom from rank 1")
    dist.barrier()
    return "unreachable"


def _tiny_model():
    torch.manual_seed(11)
    return torch.nn.Sequential(torch.nn.Linear(10, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))


def _data(n=8):
    g = torch.Generator().manual_seed(5)
    return torch.randn(n, 10, generator=g), torch.randint(0, 3, (n,), generator=g)


class _GlooEngine:
    """Stand-in for the native RCCL engine (same all_reduce/wait contract) on gloo."""

    def __init__(self):
        self.calls, self.waits = [], 0

    def all_reduce(self, t):
        import torch.distributed as dist
        self.calls.append(t.numel())
        dist.all_reduce(t)

    def wait(self):
        self.waits += 1


def _ddp_equivalence(accum, engine=False):
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.optim import FlatSGD, ParamArena
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    rank, world = dist.get_rank(), dist.get_world_size()
    x, y = _data(8 * accum)
    # reference: one process, full batch
    ref = _tiny_model()
    loss = torch.nn.functional.cross_entropy(ref(x), y)
    loss.backward()
    with torch.no_grad():
        for p in ref.parameters():
            p -= 0.1 * p.grad
    # DP: each rank gets its shard, split further into `accum` micro-batches
    m = _tiny_model()
    arena = ParamArena(list(m.named_parameters()))
    eng = _GlooEngine() if engine else "auto"
    ddp = DataParallel(m, arena, bucket_mb=0.0005, first_bucket_mb=0.0002, comm=eng)
    opt = FlatSGD(arena, lr=0.1, momentum=0.0)
    xs, ys = x[rank::world], y[rank::world]
    ddp.zero_grad()
    for i in range(accum):
        xm, ym = xs[i::accum], ys[i::accum]
        ctx = ddp.no_sync() if i < accum - 1 else torch.enable_grad()
        with ctx:
            torch.nn.functional.cross_entropy(ddp(xm), ym).backward()
    g = ddp.finish()
    opt.step(g, grad_scale=1.0 / (world * accum))
    err = max((a - b).abs().max().item() for a, b in zip(m.parameters(), ref.parameters()))
    out = {"err": err, "nbuckets": len(ddp.buckets), "comm": ddp.comm}
    if engine:
        out.update(engine_calls=len(eng.calls), engine_waits=eng.waits)
    return out


def _hvd_equivalence():
    from databricks_distributed_deep_learning_amd.parallel import hvd
    hvd.init()
    x, y = _data(8)
    ref = _tiny_model()
    torch.nn.functional.cross_entropy(ref(x), y).backward()
    with torch.no_grad():
        for p in ref.parameters():
            p -= 0.1 * p.grad
    m = _tiny_model()
    opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), named_parameters=m.named_parameters())
    hvd.broadcast_parameters(m.state_dict(), root_rank=0)
    opt.zero_grad()
    r, w = hvd.rank(), hvd.size()
    torch.nn.functional.cross_entropy(m(x[r::w]), y[r::w]).backward()
    opt.step()
    err = max((a - b).abs().max().item() for a, b in zip(m.parameters(), ref.parameters()))
    ar = hvd.allreduce(torch.tensor([float(r)]), average=True)
    ag = hvd.allgather(torch.tensor([[float(r)]]))
    bc = hvd.broadcast(torch.tensor([float(r + 5)]), root_rank=1)
    return {"err": err, "avg": ar.item(), "gather": ag.flatten().tolist(), "bcast": bc.item()}


def _train_resnet18_gloo(tmpdir):
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    cfg = get_preset("resnet18_gloo", batch_size=2, image_size=32, steps=2, warmup_steps=1,
                     checkpoint_dir=os.path.join(tmpdir, "ck"), num_classes=10)
    s = Trainer(cfg).run()
    # resume from the checkpoint written at the end of the run
    cfg2 = cfg.replace(resume=True, steps=1, warmup_steps=0, checkpoint_dir=cfg.checkpoint_dir)
    t2 = Trainer(cfg2)
    resumed_step = t2.step
    s2 = t2.run()
    return {"summary": s, "resumed_step": resumed_step, "loss2": s2["final_loss"]}


def _train_zero_checkpoint(tmpdir):
    """ZeRO-1 + checkpointing: state_dict() all-gathers the sharded state, so every rank
    must take it (a rank-0-only call deadlocks against the others' barrier)."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    cfg = get_preset("resnet18_gloo", batch_size=2, image_size=32, steps=2, warmup_steps=0, optimizer="adamw",
                     lr=1e-3, checkpoint_dir=os.path.join(tmpdir, "ckz"), checkpoint_every=1, num_classes=10,
                     zero_optimizer=True)
    t = Trainer(cfg)
    assert t.opt.shard is not None
    s = t.run()
    # compare the full (gathered) state: the local shards depend on the bucket layout, which the
    # default auto bucket policy sizes from a timed comm probe -- so pin a different layout on
    # resume on purpose (the checkpoint is layout-independent)
    before = {k: x.clone() for k, x in t.opt.state_dict().items() if torch.is_tensor(x)}
    t2 = Trainer(cfg.replace(resume=True, steps=1, bucket_mb=1.0, first_bucket_mb=0.5))
    after = {k: x for k, x in t2.opt.state_dict().items() if torch.is_tensor(x)}
    assert set(before) == set(after) == {"master", "exp_avg", "exp_avg_sq"}
    err = max((after[k] - before[k]).abs().max().item() for k in before)
    resumed = t2.step
    s2 = t2.run()
    return {"rank": dist.get_rank(), "err": err, "resumed_step": resumed, "loss": s["final_loss"],
            "loss2": s2["final_loss"]}


def _overlap_equivalence(opt_name):
    """Per-bucket optimizer updates as each all-reduce completes (finish(on_ready=...))
    == one fused step after the last all-reduce."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.optim import ParamArena
    from databricks_distributed_deep_learning_amd.optim.flat import FlatAdamW, FlatLAMB, FlatSGD
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    rank, world = dist.get_rank(), dist.get_world_size()
    cls = {"sgd": FlatSGD, "adamw": FlatAdamW, "lamb": FlatLAMB}[opt_name]
    kw = {"sgd": dict(lr=0.1, momentum=0.9, weight_decay=1e-3), "adamw": dict(lr=1e-2, weight_decay=0.01),
          "lamb": dict(lr=1e-2, weight_decay=0.01, max_grad_norm=0.0)}[opt_name]
    x, y = _data(16)
    x, y = x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]
    finals, nb = [], 0
    for overlap in (False, True):
        model = _tiny_model()
        arena = ParamArena(list(model.named_parameters()))
        ddp = DataParallel(model, arena, bucket_mb=0.0005, first_bucket_mb=0.0002)
        opt = cls(arena, **kw)
        nb = len(ddp.buckets)
        for _ in range(3):
            ddp.zero_grad()
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
            if overlap:
                opt.begin_step()
                seen = []
                ddp.finish(on_ready=lambda g, lo, hi: (seen.append((lo, hi)), opt.step_range(g, 0.5, lo, hi)))
                opt.end_step()
                assert sorted(seen) == [(b.start, b.end) for b in ddp.buckets]
            else:
                opt.step(ddp.finish(), grad_scale=0.5)
        finals.append(torch.cat([p.detach().flatten() for p in model.parameters()]))
    return {"err": (finals[0] - finals[1]).abs().max().item(), "nbuckets": nb}


def _broadcast_init_check():
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    torch.manual_seed(dist.get_rank())          # deliberately different init per rank
    m = torch.nn.Linear(4, 4)
    DataParallel(m)
    w = m.weight.detach().clone()
    dist.all_reduce(w)
    return (w / dist.get_world_size() - m.weight.detach()).abs().max().item()


# ---------------------------------------------------------------- tests
def _sync_bn_equivalence():
    """SyncBatchNorm on each rank's half batch == BatchNorm over the full batch."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.models.layers import BatchNorm2d, convert_sync_batchnorm
    rank, world = dist.get_rank(), dist.get_world_size()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 5, 5, 16, generator=g) * 2 + 0.5
    r = torch.randn(8, 5, 5, 16, generator=g)
    dy = torch.randn(8, 5, 5, 16, generator=g)
    ref = BatchNorm2d(16, relu=True)
    with torch.no_grad():
        ref.weight.copy_(torch.rand(16, generator=g) + 0.5)
    sync = BatchNorm2d(16, relu=True)
    sync.load_state_dict(ref.state_dict())
    convert_sync_batchnorm(sync)
    xr = x.clone().requires_grad_(True)
    (ref(xr, residual=r) * dy).sum().backward()
    lo, hi = rank * 8 // world, (rank + 1) * 8 // world
    xs = x[lo:hi].clone().requires_grad_(True)
    (sync(xs, residual=r[lo:hi]) * dy[lo:hi]).sum().backward()
    out_err = (sync(x[lo:hi].clone(), residual=r[lo:hi]) - ref(x.clone(), residual=r)[lo:hi]).abs().max().item()
    # parameter gradients are per-rank partials: their sum over ranks is the full-batch gradient
    gw = sync.weight.grad.clone()
    dist.all_reduce(gw)
    return {"dx": (xs.grad - xr.grad[lo:hi]).abs().max().item(),
            "dw": (gw - ref.weight.grad).abs().max().item(),
            "rm": (sync.running_mean - ref.running_mean).abs().max().item(),
            "rv": (sync.running_var - ref.running_var).abs().max().item(),
            "out": out_err}


def test_sync_batchnorm_matches_full_batch():
    out = Distributor(num_processes=2, use_gpu=False).run(_sync_bn_equivalence)
    assert max(out.values()) < 1e-4, out


def _zero_equivalence(opt_name):
    """ZeRO-1 (state sharded 1/world, params all-gathered) == replicated optimizer."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.optim import ParamArena
    from databricks_distributed_deep_learning_amd.optim.flat import FlatAdamW, FlatLAMB, FlatSGD
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    rank, world = dist.get_rank(), dist.get_world_size()
    cls = {"sgd": FlatSGD, "adamw": FlatAdamW, "lamb": FlatLAMB}[opt_name]
    kw = {"sgd": dict(lr=0.1, momentum=0.9, weight_decay=1e-3), "adamw": dict(lr=1e-2, weight_decay=0.01),
          "lamb": dict(lr=1e-2, weight_decay=0.01)}[opt_name]
    x, y = _data(16)
    x, y = x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]
    finals, state = [], []
    for shard in (None, (rank, world)):
        model = _tiny_model()
        arena = ParamArena(list(model.named_parameters()), pad_multiple=world * 64 if shard else 1)
        ddp = DataParallel(model, arena, bucket_mb=0.0005, first_bucket_mb=0.0002)
        opt = cls(arena, shard=shard, **kw)
        for _ in range(3):
            ddp.zero_grad()
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
            opt.step(ddp.finish(), grad_scale=ddp.grad_scale)
        finals.append(torch.cat([p.detach().flatten() for p in model.parameters()]))
        state.append(opt.state_numel)
        sd = opt.state_dict()          # full-arena tensors even when sharded
    err = (finals[0] - finals[1]).abs().max().item()
    return {"err": err, "state": state, "sd_master": sd["master"].numel() if "master" in sd else -1,
            "arena": arena.numel}


@pytest.mark.parametrize("opt_name", ["sgd", "adamw", "lamb"])
def test_zero1_sharded_optimizer_matches_replicated(opt_name):
    out = Distributor(num_processes=2, use_gpu=False).run(_zero_equivalence, opt_name)
    assert out["err"] < 1e-6, out
    full, sharded = out["state"]
    assert sharded * 2 == out["arena"] and full < out["arena"] + 64, out


def test_distributor_returns_rank0_value():
    out = Distributor(num_processes=2, use_gpu=False).run(_rank_info, "hello")
    assert out == {"tag": "hello", "rank": 0, "world": 2, "sum": 3.0}


def test_distributor_single_process_inline():
    assert Distributor(1, use_gpu=False, init_process_group=False).run(lambda a: a + 1, 41) == 42


def test_distributor_propagates_child_failure():
    with pytest.raises(ChildFailed) as ei:
        Distributor(num_processes=2, use_gpu=False, timeout_s=120).run(_fail_on_rank1)
    assert ei.value.rank == 1 and "boom from rank 1" in str(ei.value)


@pytest.mark.parametrize("accum", [1, 2])
def test_ddp_matches_single_process_large_batch(accum):
    out = Distributor(num_processes=2, use_gpu=False).run(_ddp_equivalence, accum)
    assert out["err"] < 1e-6, out
    assert out["nbuckets"] > 1


@pytest.mark.parametrize("accum", [1, 2])
def test_ddp_engine_contract(accum):
    """The reducer drives a comm engine (the native RCCL engine's contract): one
    all_reduce per bucket, none on no_sync micro-steps, one wait per step."""
    out = Distributor(num_processes=2, use_gpu=False).run(_ddp_equivalence, accum, True)
    assert out["err"] < 1e-6, out
    assert out["comm"] == "native"
    assert out["engine_calls"] == out["nbuckets"] and out["engine_waits"] == 1, out


def test_ddp_broadcasts_rank0_params():
    assert Distributor(num_processes=2, use_gpu=False).run(_broadcast_init_check) < 1e-7


def test_horovod_runner_and_facade():
    out = HorovodRunner(np=2, use_gpu=False).run(_hvd_equivalence)
    assert out["err"] < 1e-6
    assert out["avg"] == 0.5
    assert out["gather"] == [0.0, 1.0]
    assert out["bcast"] == 6.0


def test_notebook_train_resnet18_gloo_world2_with_resume(tmp_path):
    out = Distributor(num_processes=2, use_gpu=False, timeout_s=600).run(_train_resnet18_gloo, str(tmp_path))
    s = out["summary"]
    assert s["world_size"] == 2 and s["global_batch"] == 4
    assert s["samples_per_sec"] > 0 and s["final_loss"] == s["final_loss"]
    assert out["resumed_step"] == 3
    assert out["loss2"] == out["loss2"]


def test_zero1_checkpoint_save_and_resume_world2(tmp_path):
    out = Distributor(num_processes=2, use_gpu=False, timeout_s=600).run(_train_zero_checkpoint, str(tmp_path))
    assert out["err"] == 0.0, out
    assert out["resumed_step"] == 2, out
    assert out["loss2"] == out["loss2"], out


@pytest.mark.parametrize("opt_name", ["sgd", "adamw", "lamb"])
def test_optimizer_overlapped_with_bucket_allreduce(opt_name):
    out = Distributor(num_processes=2, use_gpu=False).run(_overlap_equivalence, opt_name)
    assert out["nbuckets"] > 1 and out["err"] < 1e-6, out


def _zero_rs_equivalence(opt_name, accum):
    """ZeRO-1 through the reducer: buckets reduce-scattered into the local gradient shard,
    sharded step, per-bucket all-gathers waited by forward pre-hooks == replicated DP."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.optim import ParamArena
    from databricks_distributed_deep_learning_amd.optim.flat import FlatAdamW, FlatLAMB, FlatSGD
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    rank, world = dist.get_rank(), dist.get_world_size()
    cls = {"sgd": FlatSGD, "adamw": FlatAdamW, "lamb": FlatLAMB}[opt_name]
    kw = {"sgd": dict(lr=0.1, momentum=0.9, weight_decay=1e-3), "adamw": dict(lr=1e-2, weight_decay=0.01),
          "lamb": dict(lr=1e-2, weight_decay=0.01)}[opt_name]
    x, y = _data(16 * accum)
    x, y = x[rank::world], y[rank::world]
    finals, info = [], {}
    for shard in (False, True):
        torch.manual_seed(11)
        model = torch.nn.Sequential(torch.nn.Linear(10, 96), torch.nn.Tanh(), torch.nn.Linear(96, 64),
                                    torch.nn.Tanh(), torch.nn.Linear(64, 3))
        arena = ParamArena(list(model.named_parameters()), pad_multiple=world * 64 if shard else 1)
        ddp = DataParallel(model, arena, bucket_mb=0.004, first_bucket_mb=0.001, shard=shard,
                           accumulate_fp32=accum > 1)
        opt = cls(arena, shard=(rank, world, ddp.shard_groups()) if shard else None, **kw)
        if shard:
            opt.gather_fn = ddp.gather_params
            info = {"nbuckets": len(ddp.buckets), "local": opt.state_numel, "arena": arena.numel,
                    "straddle": sum(len(v) > 1 for v in ddp._entry_buckets.values())}
        for _ in range(3):
            ddp.zero_grad()
            for i in range(accum):
                ctx = ddp.no_sync() if i < accum - 1 else torch.enable_grad()
                with ctx:
                    torch.nn.functional.cross_entropy(ddp(x[i::accum]), y[i::accum]).backward()
            g = ddp.finish()
            if shard:
                assert g.numel() == opt.state_numel
            opt.step(g, grad_scale=1.0 / (world * accum))
        ddp.wait_params()
        finals.append(torch.cat([p.detach().flatten() for p in model.parameters()]))
        sd = opt.state_dict()
    info["err"] = (finals[0] - finals[1]).abs().max().item()
    info["sd"] = sd["master"].numel()
    return info


@pytest.mark.parametrize("opt_name,accum", [("sgd", 1), ("adamw", 2), ("lamb", 1)])
def test_zero1_reduce_scatter_matches_replicated(opt_name, accum):
    out = Distributor(num_processes=2, use_gpu=False).run(_zero_rs_equivalence, opt_name, accum)
    assert out["err"] < 1e-5, out
    assert out["nbuckets"] > 1 and out["local"] * 2 == out["arena"] and out["sd"] == out["arena"], out


# ---------------------------------------------------------------- comm probe / bucket policy
def _probe_and_buckets():
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.parallel.comm import auto_buckets, probe_allreduce
    eng = _GlooEngine()
    probe = probe_allreduce(eng, "cpu", sizes_mb=(0.25, 1, 4), iters=3, dtype=torch.float32)
    first, bucket = auto_buckets(probe, total_mb=200.0)
    return {"probe": probe, "first": first, "bucket": bucket, "calls": len(eng.calls), "world": dist.get_world_size()}


def test_comm_probe_drives_auto_buckets_gloo():
    out = Distributor(num_processes=2, use_gpu=False).run(_probe_and_buckets)
    assert out["calls"] == 3 * 4 and [p["mb"] for p in out["probe"]] == [0.25, 1.0, 4.0], out
    assert all(p["ms"] > 0 and p["busbw_gbs"] > 0 for p in out["probe"]), out
    assert 1.0 <= out["first"] <= out["bucket"] / 2 + 1e-9 and 4.0 <= out["bucket"] <= 64.0, out


def test_auto_buckets_from_latency_bandwidth_model():
    from databricks_distributed_deep_learning_amd.parallel.comm import auto_buckets, fit_latency_bandwidth
    # t = 0.02 ms + S / beta with alpha * beta = 2 MiB (~105 GB/s): 16 MB buckets, 4 MB first bucket
    beta = 2 ** 21 / 0.02
    probe = [{"mb": mb, "ms": 0.02 + mb * 2 ** 20 / beta} for mb in (1, 4, 16, 64)]
    a, b = fit_latency_bandwidth(probe)
    assert abs(a - 0.02) < 1e-6 and abs(b / beta - 1) < 1e-6
    assert auto_buckets(probe, total_mb=218.0) == (4.0, 16.0)
    # a small model caps buckets at a quarter of its gradient (>= 4 MB)
    assert auto_buckets(probe, total_mb=20.0) == (2.5, 5.0)
    # latency-free links: floor of 4 MB buckets, 1 MB first bucket
    flat = [{"mb": mb, "ms": mb * 2 ** 20 / beta} for mb in (1, 4, 16, 64)]
    assert auto_buckets(flat, total_mb=500.0) == (1.0, 4.0)


def test_watchdog_fails_engine_within_seconds():
    import time
    from databricks_distributed_deep_learning_amd.parallel.comm import CommWatchdog

    class Eng:
        def __init__(self):
            self.err, self.failed, self.polls = None, None, 0

        def poll(self):
            self.polls += 1
            return self.err

        def fail(self, reason):
            self.failed = reason

    e = Eng()
    wd = CommWatchdog(e, interval=0.02)
    time.sleep(0.1)
    assert e.failed is None and e.polls > 1
    t0 = time.time()
    e.err = "RCCL asynchronous error 6 on rank 1"
    while e.failed is None and time.time() - t0 < 5:
        time.sleep(0.01)
    assert e.failed == e.err and time.time() - t0 < 2
    wd.stop()
    assert wd.reason == e.err


def _split_bucket_equivalence(opt_name):
    """A tensor larger than a bucket is cut into bucket-sized pieces (BERT's word embedding):
    the pieces all-reduce separately and the per-bucket optimizer ranges still give the same
    update as replicated full-batch training."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.optim import ParamArena
    from databricks_distributed_deep_learning_amd.optim.flat import FlatAdamW, FlatSGD
    from databricks_distributed_deep_learning_amd.parallel import DataParallel
    rank, world = dist.get_rank(), dist.get_world_size()
    cls = {"sgd": FlatSGD, "adamw": FlatAdamW}[opt_name]
    finals, layout = [], None
    for split in (False, True):
        torch.manual_seed(3)
        emb = torch.nn.Embedding(600, 64)          # 38400 elements: > 2 x 16384-element buckets
        head = torch.nn.Linear(64, 5)
        model = torch.nn.ModuleDict({"emb": emb, "head": head})
        arena = ParamArena(list(model.named_parameters()))
        ddp = DataParallel(model, arena, bucket_mb=16384 * 4 / 2 ** 20, first_bucket_mb=0.001, split_tensors=split)
        opt = cls(arena, lr=0.05)
        ids = torch.randint(0, 600, (8, 12), generator=torch.Generator().manual_seed(7 + rank))
        for _ in range(2):
            ddp.zero_grad()
            head(emb(ids).mean(1)).square().mean().backward()
            opt.begin_step()
            ddp.finish(on_ready=lambda g, lo, hi: opt.step_range(g, 1.0 / world, lo, hi))
            opt.end_step()
        finals.append(torch.cat([p.detach().flatten() for p in model.parameters()]))
        if split:
            layout = [(b.start, b.end, b.entry_ids) for b in ddp.buckets]
    return {"err": (finals[0] - finals[1]).abs().max().item(), "layout": layout}


@pytest.mark.parametrize("opt_name", ["sgd", "adamw"])
def test_split_tensor_buckets_match(opt_name):
    out = Distributor(num_processes=2, use_gpu=False).run(_split_bucket_equivalence, opt_name)
    pieces = [b for b in out["layout"] if len(b[2]) == 1 and b[1] - b[0] >= 8192]
    assert len(pieces) >= 2, out["layout"]
    assert all((b[0] - pieces[0][0]) % 8192 == 0 for b in pieces), out["layout"]
    assert out["err"] < 1e-6, out


# ---------------------------------------------------------------- bf16 vs fp32 gradient payloads
def _ring_sum_bf16(chunks):
    """What an n-rank RCCL ring all-reduce computes for a bf16 payload: the reduce-scatter walks
    each chunk through the ranks in ring order, every hop adding in fp32 and storing the running
    sum as bf16 (n - 1 roundings), then the all-gather copies the result unchanged."""
    acc = chunks[0].to(torch.bfloat16)
    for c in chunks[1:]:
        acc = (acc.float() + c.to(torch.bfloat16).float()).to(torch.bfloat16)
    return acc.float()


def _bert_grad_reduce_error():
    """Each of 8 ranks computes real BERT-base-architecture gradients (bf16 model, its own
    micro-batch; 2 encoder layers to keep 8 CPU processes fast) -- the payload the data-parallel
    reducer ships.  Rank 0 compares the summed gradient of an fp32 payload, gloo's own bf16
    all-reduce and an RCCL-ring bf16 emulation against an fp64 sum."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.models.bert import bert_base
    ops.set_native_mode("off")
    r, n = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(0)
    m = bert_base(num_labels=2, dropout=0.0, num_hidden_layers=2, vocab_size=4096).to(torch.bfloat16)
    g = torch.Generator().manual_seed(100 + r)
    ids = torch.randint(0, 4096, (4, 64), generator=g)
    labels = torch.randint(0, 2, (4,), generator=g)
    loss, _ = m(ids, None, None, labels)
    loss.backward()
    grad = torch.cat([p.grad.reshape(-1) for p in m.parameters() if p.grad is not None])   # bf16
    # fp32 payload (what grad_reduce_dtype=fp32 ships) and bf16 payload through gloo
    g32 = grad.float().clone()
    dist.all_reduce(g32)
    try:
        g16 = grad.clone()
        dist.all_reduce(g16)
        g16 = g16.float()
    except RuntimeError:              # gloo without bf16 sums: the ring emulation below only
        g16 = None
    every = [torch.empty_like(grad) for _ in range(n)]
    dist.all_gather(every, grad)
    if r != 0:
        return None
    ref = torch.stack([e.double() for e in every]).sum(0)
    ring = _ring_sum_bf16([e for e in every])

    def rel(x):
        return float((x.double() - ref).norm() / ref.norm())
    once = rel(ref.to(torch.bfloat16))          # the unavoidable part: one rounding of the exact sum
    return {"fp32": rel(g32), "gloo_bf16": None if g16 is None else rel(g16), "ring_bf16": rel(ring),
            "round_once": once, "numel": grad.numel()}


def test_bf16_gradient_reduce_error_world8():
    """Gradient-reduce payload precision at world 8.  The default payload is
    the arena dtype (bf16): an 8-rank ring rounds every running sum to bf16 seven times.  Measured
    on real BERT gradients: the ring's relative error (L2, whole gradient) is a small multiple of a
    single bf16 rounding of the exact sum and well under 1 % -- far below the minibatch gradient
    noise the optimizer sees -- so the bf16 payload (half the xGMI bytes) stays the default;
    ``grad_reduce_dtype=fp32`` is the switch for anyone who wants the exact sum."""
    out = Distributor(num_processes=8, use_gpu=False, timeout_s=600).run(_bert_grad_reduce_error)
    assert out["fp32"] < 1e-6, out
    assert out["ring_bf16"] < 8 * out["round_once"], out
    assert out["ring_bf16"] < 0.01, out
    if out["gloo_bf16"] is not None:
        assert out["gloo_bf16"] < 0.01, out
    print("bf16 vs fp32 reduce error (8 ranks):", out)


def _auto_bucket_policy_trainer():
    """Trainer with bucket_mb = 0 ("auto"): probe -> auto_buckets -> bucket layout, end to end."""
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.parallel.comm import auto_buckets
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    cfg = get_preset("resnet18_gloo", batch_size=2, image_size=32, steps=1, warmup_steps=0, num_classes=10,
                     bucket_mb=0.0, log_every=0)
    tr = Trainer(cfg)
    s = tr.run()
    esz = torch.empty((), dtype=tr.ddp.reduce_dtype).element_size()
    total = tr.arena.numel * esz / 2 ** 20
    want = auto_buckets(s["comm_probe"], total) if s.get("comm_probe") else None
    # the layout those sizes give (the reducer's own rule), to compare with the one it built
    layout = [(b.end - b.start) * esz / 2 ** 20 for b in tr.ddp._build_buckets(want[1], want[0])] if want else None
    out = {"policy": s["bucket_policy"], "probe": s.get("comm_probe"), "buckets": s["buckets_mb"],
           "want": want, "layout": layout, "total": total,
           "world": dist.get_world_size(), "rank": dist.get_rank(), "loss": s["final_loss"]}
    tr.close()
    return out


def _gather_all(fn):
    import torch.distributed as dist
    out = fn()
    allv = [None] * dist.get_world_size()
    dist.all_gather_object(allv, out)
    return allv


def _auto_bucket_policy_all_ranks():
    return _gather_all(_auto_bucket_policy_trainer)


def test_auto_bucket_policy_end_to_end_world8():
    """8 gloo ranks through the Trainer with the default "auto" bucket size:
    the startup all-reduce probe runs (over the process group: no native engine on the CPU),
    every rank derives the SAME (first, bucket) sizes from it (the probe's per-size times are
    the max over ranks -- per-rank timings would otherwise give ranks different bucket layouts,
    i.e. mismatched all-reduces), and the reducer's buckets follow those sizes."""
    ranks = Distributor(num_processes=8, use_gpu=False).run(_auto_bucket_policy_all_ranks)
    assert len(ranks) == 8 and sorted(r["rank"] for r in ranks) == list(range(8))
    r0 = ranks[0]
    assert r0["world"] == 8 and r0["policy"]["source"] == "probe", r0["policy"]
    assert [p["mb"] for p in r0["probe"]] == [0.25, 1.0, 4.0]
    first, bucket = r0["want"]
    assert (r0["policy"]["first_bucket_mb"], r0["policy"]["bucket_mb"]) == (first, bucket)
    for r in ranks[1:]:
        assert r["probe"] == r0["probe"] and r["policy"] == r0["policy"] and r["buckets"] == r0["buckets"], r
    b = r0["buckets"]
    assert abs(sum(b) - r0["total"]) < 0.005 * len(b) + 1e-3, (b, r0["total"])   # (2-decimal MB)
    # the reducer's buckets are the layout of exactly those sizes (whole tensors per bucket, closed
    # by the tensor reaching the cap; tensors above a bucket cut into pieces of their own)
    assert [round(x, 2) for x in b] == [round(x, 2) for x in r0["layout"]], (b, r0["layout"])
    assert all(x < 2 * bucket + 0.01 for x in b), (b, bucket)
    assert all(abs(r["loss"] - r0["loss"]) < 1e-6 for r in ranks)
