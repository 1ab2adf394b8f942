"""Native RCCL comm engine (csrc/runtime/comm.cpp) on one GPU: communicator
bring-up over a torch.distributed store, stream ordering, every collective at
world size 1, and the DataParallel reducer driving it.  (Multi-rank RCCL needs
one GPU per rank; the 8-GPU path runs in the driver's scaling bench.)"""
import os

import pytest
import torch
import torch.distributed as dist

from conftest import gpu_device

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.parallel.dist import _free_port as free_port
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(free_port())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    yield dev
    dist.destroy_process_group()


def test_native_collectives(pg):
    from databricks_distributed_deep_learning_amd.parallel.comm import NativeComm
    c = NativeComm()
    x = torch.randn(1 << 20, device=pg, dtype=torch.bfloat16)
    want = x.clone()
    # producer kernel right before the collective: the engine must order after it
    x.mul_(2.0)
    c.all_reduce(x)
    c.wait()
    torch.testing.assert_close(x, want * 2)
    ys = [torch.randn(n, device=pg) for n in (7, 4096, 123457)]
    ref = [y.clone() for y in ys]
    c.all_reduce_many(ys, average=True)
    c.wait()
    for y, r in zip(ys, ref):
        torch.testing.assert_close(y, r)
    b = torch.arange(100, device=pg, dtype=torch.float32)
    c.broadcast(b)
    rs = torch.empty(100, device=pg)
    c.reduce_scatter(b, rs)
    ag = torch.empty(100, device=pg)
    c.all_gather(rs, ag)
    c.wait()
    torch.testing.assert_close(ag, torch.arange(100, device=pg, dtype=torch.float32))
    assert c.collectives_launched >= 4
    c.synchronize()
    c.close()


def test_reducer_native_engine(pg):
    from databricks_distributed_deep_learning_amd.models import resnet18
    from databricks_distributed_deep_learning_amd.optim.arena import ParamArena
    from databricks_distributed_deep_learning_amd.parallel.ddp import DataParallel
    torch.manual_seed(0)
    m = resnet18(num_classes=10).to(pg)
    ddp = DataParallel(m, ParamArena(list(m.named_parameters())), bucket_mb=4, first_bucket_mb=1, comm="native")
    assert ddp.comm == "native" and len(ddp.buckets) > 2
    x = torch.randn(4, 64, 64, 3, device=pg)
    loss = m(x).float().square().mean()
    loss.backward()
    g = ddp.finish()
    assert torch.isfinite(g).all() and g.abs().sum() > 0
    # reference gradients through autograd without the reducer's arena
    m2 = resnet18(num_classes=10).to(pg)
    m2.load_state_dict(m.state_dict())
    m2(x).float().square().mean().backward()
    grads2 = {n: p.grad for n, p in m2.named_parameters()}
    ref = torch.cat([grads2[e.name].reshape(-1) for e in ddp.arena.entries])
    got = torch.cat([g[e.offset:e.offset + e.numel] for e in ddp.arena.entries])
    assert ((got.float() - ref.float()).abs().max() / ref.abs().max()).item() < 1e-3


@pytest.mark.parametrize("fused_stats", [False, True])
def test_sync_batchnorm_native_world1(pg, fused_stats):
    """SyncBatchNorm's split native path (partials -> one row -> all-reduce -> finalize /
    apply with the global count) at world size 1 must equal the fused single-GPU path,
    with statistics from the BN's own pass or from the conv GEMM epilogue."""
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.ops.bridge import BNStats
    torch.manual_seed(9)
    x = torch.randn(16, 30, 30, 64, device=pg).to(torch.bfloat16)
    w = (torch.randn(128, 3, 3, 64, device=pg) * 0.05).to(torch.bfloat16)
    g = (torch.rand(128, device=pg) + 0.5).to(torch.bfloat16)
    b = (torch.randn(128, device=pg) * 0.1).to(torch.bfloat16)
    dy = torch.randn(16, 30, 30, 128, device=pg).to(torch.bfloat16)
    outs = []
    for group in (None, dist.group.WORLD):
        xs, gs, bs = (t.clone().requires_grad_(True) for t in (x, g, b))
        rm, rv = torch.zeros(128, device=pg), torch.ones(128, device=pg)
        st = BNStats() if fused_stats else None
        from databricks_distributed_deep_learning_amd.ops import _native_conv as NC
        saved, NC.STATS_MIN_K = NC.STATS_MIN_K, 0
        try:
            y = ops.conv2d(xs, w, 1, 1, bn_stats=st)
        finally:
            NC.STATS_MIN_K = saved
        z = ops.batch_norm(y, gs, bs, rm, rv, True, 0.1, 1e-5, True, None, stats=st, group=group)
        z.backward(dy)
        outs.append((z.float(), xs.grad.float(), gs.grad.float(), bs.grad.float(), rm, rv))
    for a, c in zip(outs[0], outs[1]):
        torch.testing.assert_close(a, c, rtol=2e-2, atol=2e-2)


def test_sync_batchnorm_rides_the_reducer_engine(pg):
    """With the reducer's native engine active, SyncBatchNorm's statistic all-reduces go
    through that same communicator / comm stream (one RCCL communicator carries every
    in-backward collective) and give the same result as the torch process group."""
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.parallel import comm as C
    torch.manual_seed(4)
    x = torch.randn(8, 14, 14, 64, device=pg).to(torch.bfloat16)
    g = (torch.rand(64, device=pg) + 0.5).to(torch.bfloat16)
    b = (torch.randn(64, device=pg) * 0.1).to(torch.bfloat16)
    dy = torch.randn(8, 14, 14, 64, device=pg).to(torch.bfloat16)
    eng = C.NativeComm()
    outs = []
    try:
        for active in (None, eng):
            C.set_active(active)
            before = eng.collectives_launched
            xs, gs, bs = (t.clone().requires_grad_(True) for t in (x, g, b))
            rm, rv = torch.zeros(64, device=pg), torch.ones(64, device=pg)
            z = ops.batch_norm(xs, gs, bs, rm, rv, True, 0.1, 1e-5, True, None, group=dist.group.WORLD)
            z.backward(dy)
            torch.cuda.synchronize()
            outs.append((z.float(), xs.grad.float(), gs.grad.float(), rm, rv))
            # forward statistics + backward coefficients: two all-reduces on the engine when active
            assert eng.collectives_launched - before == (2 if active is not None else 0)
    finally:
        C.set_active(None)
        eng.close()
    for a, c in zip(outs[0], outs[1]):
        torch.testing.assert_close(a, c, rtol=1e-2, atol=1e-2)


def test_reducer_native_per_bucket_ready(pg):
    """finish(on_ready=...) with the native engine: the compute stream waits for each
    bucket's own all-reduce (wait_upto on the engine's completion ring), and a
    range-stepped optimizer over those callbacks equals one fused step."""
    from databricks_distributed_deep_learning_amd.models import resnet18
    from databricks_distributed_deep_learning_amd.optim import FlatSGD
    from databricks_distributed_deep_learning_amd.optim.arena import ParamArena
    from databricks_distributed_deep_learning_amd.parallel.ddp import DataParallel
    x = torch.randn(4, 64, 64, 3, device=pg)
    finals = []
    # fp32 model: the convolutions run on the reference path (MIOpen), whose weight-gradient
    # algorithm choice is not deterministic across runs -- pin it, and compare with a
    # tolerance far below what a bucket stepped out of order would change
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    for overlap in (False, True):
        torch.manual_seed(0)
        m = resnet18(num_classes=10).to(pg)
        arena = ParamArena(list(m.named_parameters()))
        ddp = DataParallel(m, arena, bucket_mb=4, first_bucket_mb=1, comm="native")
        opt = FlatSGD(arena, lr=0.05, momentum=0.9)
        for _ in range(2):
            ddp.zero_grad()
            m(x).float().square().mean().backward()
            if overlap:
                opt.begin_step()
                seqs = []
                ddp.finish(on_ready=lambda g, lo, hi: (seqs.append(lo), opt.step_range(g, 1.0, lo, hi)))
                opt.end_step()
                assert len(seqs) == len(ddp.buckets) > 2
            else:
                opt.step(ddp.finish())
        torch.cuda.synchronize()
        finals.append(arena.flat.float().clone())
    torch.backends.cudnn.deterministic = det
    torch.testing.assert_close(finals[0], finals[1], atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("preset,over", [
    ("resnet50_ddp", dict(model="resnet18", batch_size=8, image_size=64, num_classes=10)),
    ("bert_base_ddp", dict(batch_size=4, seq_len=64)),
])
def test_eager_optimizer_matches_post_backward_step(pg, preset, over):
    """Optimizer updates issued per bucket DURING backward on a side stream
    (DataParallel.set_eager) give the same parameters and state as one step after backward."""
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    finals = []
    for eager in (True, False):
        cfg = get_preset(preset, steps=3, warmup_steps=0, log_every=0, eager_optimizer=eager, **over)
        t = Trainer(cfg)
        assert t.eager_optimizer == eager
        t.run()
        torch.cuda.synchronize()
        st = [t.arena.flat.float().clone()] + [v.float().clone() for v in t.opt._state_tensors().values()]
        finals.append(st)
        del t
    for a, b in zip(*finals):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)


def test_engine_sequence_numbers_and_inplace_all_gather(pg):
    """ZeRO-1's engine contract at world 1: reduce-scatter / all-gather / all-reduce share one
    increasing sequence, wait_upto(seq) orders the compute stream after THAT collective, and an
    all-gather whose send buffer is its own slice of recv (the in-place flat[lo:hi] ->
    flat[a:b] gather of DataParallel.gather_params) leaves the data intact."""
    from databricks_distributed_deep_learning_amd.parallel.comm import NativeComm
    c = NativeComm(timeout_s=0)
    flat = torch.randn(4096, device=pg, dtype=torch.bfloat16)
    want = flat.clone()
    s1 = c.reduce_scatter(flat[:1024].clone(), torch.empty(1024, device=pg, dtype=torch.bfloat16))
    s2 = c.all_gather(flat[1024:2048], flat[1024:2048])       # send is recv itself (world 1: its own slice)
    s3 = c.all_reduce(flat[2048:])
    assert 0 < s1 < s2 < s3
    c.wait_upto(s2)
    torch.testing.assert_close(flat[1024:2048], want[1024:2048])
    c.wait_upto(s3)
    torch.cuda.synchronize()
    torch.testing.assert_close(flat, want)
    # per-collective device time from the engine's start / done events
    assert all(c.collective_ms(s) >= 0 for s in (s1, s2, s3))
    assert c.collective_ms(s3 + 5) == -1.0
    c.close()


def test_watchdog_aborts_on_async_error(pg):
    """An RCCL asynchronous error (injected: what a peer failure looks like) is seen by the
    watchdog within seconds; the communicator is aborted and the next call raises CommError."""
    import time
    from databricks_distributed_deep_learning_amd.parallel.comm import CommError, NativeComm
    c = NativeComm(timeout_s=30, poll_s=0.05)
    x = torch.ones(1024, device=pg)
    c.all_reduce(x)
    c.wait()
    torch.cuda.synchronize()
    assert c.poll() is None and c.failed is None
    t0 = time.time()
    c.inject_error(6)            # ncclRemoteError
    while c.failed is None and time.time() - t0 < 10:
        time.sleep(0.02)
    assert c.failed and "asynchronous error 6" in c.failed, c.failed
    assert time.time() - t0 < 5
    with pytest.raises(CommError):
        c.all_reduce(x)
    c.close()


def test_watchdog_aborts_blocked_enqueue(pg):
    """An enqueue that blocks inside the engine (held API lock: RCCL connection setup to a dead
    peer) is seen by the watchdog as a pending collective and aborted: the watchdog's calls never
    wait for the API lock, the blocked call returns CommError, and close() does not hang."""
    import threading
    import time
    from databricks_distributed_deep_learning_amd.parallel.comm import CommError, NativeComm
    c = NativeComm(timeout_s=0.5, poll_s=0.05)
    x = torch.ones(4096, device=pg)
    c.all_reduce(x)
    c.wait()
    torch.cuda.synchronize()
    c.stall_next_enqueue(4000)
    err = []

    def enqueue():
        try:
            c.all_reduce(x)
        except CommError as e:
            err.append(str(e))

    t = threading.Thread(target=enqueue)
    t0 = time.time()
    t.start()
    while c.failed is None and time.time() - t0 < 10:
        time.sleep(0.02)
    # aborted while the enqueue was still blocked (it blocks for 4 s)
    assert c.failed and "unfinished after" in c.failed, c.failed
    assert time.time() - t0 < 3.5
    t.join(timeout=10)
    assert not t.is_alive() and err, err
    with pytest.raises(CommError):
        c.broadcast(x)
    c.close()


def test_abort_while_enqueue_holds_communicator(pg):
    """the abort must never free the communicator under a thread still using it.  In
    non-blocking mode the stalled enqueue is an RCCL call answering ncclInProgress, polled WHILE
    the enqueue holds the communicator (in-flight guard): the abort lands in the middle of it,
    waits for the poller to leave (it checks the abort flag between polls) and only then calls
    ncclCommAbort -- the enqueue returns CommError within a fraction of its 4 s stall, close()
    returns, and a second communicator on the same device works afterwards."""
    import threading
    import time
    from databricks_distributed_deep_learning_amd.parallel.comm import CommError, NativeComm
    c = NativeComm(timeout_s=0)
    assert c.nonblocking, "RCCL without ncclCommInitRankConfig: blocking mode"
    x = torch.ones(4096, device=pg)
    c.all_reduce(x)
    c.wait()
    torch.cuda.synchronize()
    c.stall_next_enqueue(4000)
    err, done_at = [], []

    def enqueue():
        try:
            c.all_reduce(x)
        except CommError as e:
            err.append(str(e))
        done_at.append(time.time())

    t = threading.Thread(target=enqueue)
    t.start()
    time.sleep(0.3)                       # the enqueue is now polling with the communicator held
    assert t.is_alive()
    t0 = time.time()
    c.fail("test abort during an enqueue")
    t_abort = time.time() - t0
    t.join(timeout=10)
    assert not t.is_alive() and err, err
    assert t_abort < 1.0 and done_at[0] - t0 < 1.0, (t_abort, done_at[0] - t0)
    c.close(abort=True)
    c2 = NativeComm(timeout_s=0)
    y = torch.full((1024,), 2.0, device=pg)
    c2.all_reduce(y)
    c2.wait()
    torch.cuda.synchronize()
    assert float(y[0]) == 2.0
    c2.close()


def test_engine_probe_and_bucket_timings(pg):
    """The startup probe runs on the engine, and the reducer reports per-bucket ring times of
    the last step (world 1: every number exists, bus bandwidth is 0 by the 2(n-1)/n factor)."""
    from databricks_distributed_deep_learning_amd.models import resnet18
    from databricks_distributed_deep_learning_amd.optim.arena import ParamArena
    from databricks_distributed_deep_learning_amd.parallel.comm import NativeComm, auto_buckets, probe_allreduce
    from databricks_distributed_deep_learning_amd.parallel.ddp import DataParallel
    c = NativeComm(timeout_s=0)
    probe = probe_allreduce(c, pg, sizes_mb=(1, 4), iters=3, world=1)
    assert [p["mb"] for p in probe] == [1.0, 4.0] and all(p["ms"] > 0 for p in probe)
    first, bucket = auto_buckets(probe, 44.0)
    assert 1.0 <= first <= bucket <= 64.0
    torch.manual_seed(0)
    m = resnet18(num_classes=10).to(pg)
    ddp = DataParallel(m, ParamArena(list(m.named_parameters())), bucket_mb=bucket, first_bucket_mb=first, comm=c)
    m(torch.randn(2, 32, 32, 3, device=pg)).float().square().mean().backward()
    ddp.finish()
    torch.cuda.synchronize()
    t = ddp.bucket_timings()
    assert len(t) == len(ddp.buckets) and all(r["ms"] is not None and r["ms"] >= 0 for r in t), t
    ddp.close()
