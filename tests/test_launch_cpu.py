"""Launch, fault-handling, tuning-agreement and resume behaviour on CPU / gloo (world 2).

Covers: bench.py launching its own ranks + the 1/2 scaling sweep (benchmarks/scaling.py),
ranks agreeing on GEMM kernel plans, Horovod ``backward_passes_per_step``, notebook-defined
functions shipped by ``Distributor`` (cloudpickle), an injected rank failure surfacing as
``ChildFailed`` through ``train()``, and bit-identical resume (RNG + loader position).
"""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch

from databricks_distributed_deep_learning_amd.parallel import ChildFailed, Distributor, HorovodRunner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", CUDA_VISIBLE_DEVICES="")


def test_bench_self_launch_and_scaling_sweep(tmp_path):
    """``bench.py --gpus 2`` without torchrun runs 2 ranks (n_gpus == 2), and the sweep
    reports both N with an efficiency computed against N = 1."""
    out = tmp_path / "scaling.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "scaling.py"), "--ns", "1,2",
                        "--max-visible", "2", "--backend", "gloo", "--model", "resnet50", "--steps", "1",
                        "--warmup", "1", "--out", str(out), "--", "--batch", "1"],
                       env=ENV, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    data = json.loads(out.read_text())
    recs = {rec["n_gpus"]: rec for rec in data["records"]}
    assert set(recs) == {1, 2}
    assert recs[2]["config"]["parallelism"] == "dp2" and recs[2]["config"]["global_batch"] == 2
    eff = data["summary"]["efficiency"]
    assert eff["1"]["efficiency"] == 1.0 and eff["2"]["efficiency"] > 0


def _agree():
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.ops import _native_gemm as g
    r = dist.get_rank()
    # rank 0 measured "small" faster, rank 1 "big" by a hair: pooled, "small" wins on both
    g._timings.clear()
    g._tuned.clear()
    g._timings["k1"] = {("big", 1): 1.00 + 0.5 * (r == 0), ("small", 1): 1.20 - 0.4 * (r == 0)}
    g._tuned["k1"] = ("small", 1) if r == 0 else ("big", 1)
    g._timings["k2"] = {("narrow", 2): 2.0, ("small", 1): 1.0 + r}
    g._tuned["k2"] = ("small", 1) if r == 0 else ("narrow", 2)
    changed = g.agree_across_ranks()
    return {"rank": r, "tuned": dict(g._tuned), "changed": changed}


def _agree_all():
    import torch.distributed as dist
    out = _agree()
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, (out["tuned"], out["changed"]))
    return got


def test_ranks_agree_on_gemm_plans():
    res = Distributor(num_processes=2, use_gpu=False).run(_agree_all)
    plans = [r[0] for r in res]
    assert plans[0] == plans[1], plans
    assert plans[0]["k1"] == ("small", 1)          # 1.5 + 1.0  vs  0.8 + 1.2 -> small (2.0 < 2.5)
    assert plans[0]["k2"] == ("small", 1)          # 1.0 + 2.0 = 3.0 < 4.0
    # rank 0 already ran "small" on both, rank 1 "big" / "narrow": both ranks must report the
    # same count (a caller re-runs a warm-up step on every rank or on none)
    assert res[0][1] == res[1][1] == 2, res


def _hvd_passes(pause):
    """backward_passes_per_step=2: gradients of two micro-batches accumulate locally and are
    all-reduced once (a pause between the passes must not matter)."""
    from databricks_distributed_deep_learning_amd.parallel import hvd
    hvd.init()
    torch.manual_seed(11)
    ref = torch.nn.Sequential(torch.nn.Linear(10, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    torch.manual_seed(11)
    m = torch.nn.Sequential(torch.nn.Linear(10, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    g = torch.Generator().manual_seed(5)
    x, y = torch.randn(16, 10, generator=g), torch.randint(0, 3, (16,), generator=g)
    r, w = hvd.rank(), hvd.size()
    # reference: the four micro-batch gradients summed (2 ranks x 2 passes), averaged over ranks
    for k in range(2 * w):
        torch.nn.functional.cross_entropy(ref(x[4 * k:4 * k + 4]), y[4 * k:4 * k + 4]).backward()
    opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), named_parameters=m.named_parameters(),
                                   backward_passes_per_step=2, bucket_mb=0.0002)
    opt.zero_grad()
    for k in range(2):
        mb = 2 * r + k
        torch.nn.functional.cross_entropy(m(x[4 * mb:4 * mb + 4]), y[4 * mb:4 * mb + 4]).backward()
        if pause:
            time.sleep(0.5)
    opt.synchronize()
    err = max((pm.grad - pr.grad / w).abs().max().item() for pm, pr in zip(m.parameters(), ref.parameters()))
    return err


@pytest.mark.parametrize("pause", [False, True])
def test_horovod_backward_passes_per_step(pause):
    assert HorovodRunner(np=2, use_gpu=False).run(_hvd_passes, pause=pause) < 1e-6


def test_distributor_ships_main_defined_function(tmp_path):
    """A train_fn defined in a script's ``__main__`` (as in a notebook cell) runs at world 2."""
    script = tmp_path / "nb.py"
    script.write_text(textwrap.dedent("""
        import torch, torch.distributed as dist
        from databricks_distributed_deep_learning_amd.parallel import Distributor

        SCALE = 7.0

        def train_fn(base):
            t = torch.tensor([float(dist.get_rank() + 1)])
            dist.all_reduce(t)
            return {"val": base + SCALE * t.item(), "world": dist.get_world_size()}

        if __name__ == "__main__":
            print("RESULT", Distributor(num_processes=2, use_gpu=False).run(train_fn, 1.0))
    """))
    r = subprocess.run([sys.executable, str(script)], env=ENV, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "RESULT {'val': 22.0, 'world': 2}" in r.stdout


def _train_with_fault():
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.training.loop import train
    cfg = get_preset("resnet18_gloo", batch_size=2, image_size=32, steps=4, warmup_steps=0, num_classes=10,
                     fault_rank=1, fault_step=1)
    return train(cfg)


def test_injected_fault_surfaces_through_train():
    t0 = time.time()
    with pytest.raises(ChildFailed) as ei:
        Distributor(num_processes=2, use_gpu=False, timeout_s=300).run(_train_with_fault)
    assert ei.value.rank == 1 and "InjectedFault" in str(ei.value)
    assert time.time() - t0 < 120


def _resume_bitwise(tmpdir):
    from databricks_distributed_deep_learning_amd.config import TrainConfig
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    base = TrainConfig(model="bert_tiny", batch_size=2, seq_len=16, num_classes=2, dtype="fp32", optimizer="adamw",
                       lr=1e-3, backend="gloo", native="off", dropout=0.1, warmup_steps=0, log_every=0,
                       synthetic_pool=3, pad_fraction=0.5)
    t = Trainer(base.replace(steps=4))
    t.run()
    full = torch.cat([p.detach().flatten() for p in t.model.parameters()])
    ck = os.path.join(tmpdir, "ck")
    t1 = Trainer(base.replace(steps=2, checkpoint_dir=ck))
    t1.run()
    t2 = Trainer(base.replace(steps=2, checkpoint_dir=ck, resume=True))
    assert t2.step == 2 and t2.loader._i == t1.loader._i
    s2 = t2.run()
    resumed = torch.cat([p.detach().flatten() for p in t2.model.parameters()])
    return {"err": (full - resumed).abs().max().item(), "phases": s2["phases_ms"]}


def test_resume_is_bit_identical(tmp_path):
    out = Distributor(num_processes=2, use_gpu=False, timeout_s=600).run(_resume_bitwise, str(tmp_path))
    assert out["err"] == 0.0, out
    assert {"fwd_ms", "bwd_ms"} <= set(out["phases"]), out


def _replicas(corrupt):
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.parallel import ReplicaDivergence
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    cfg = get_preset("resnet18_gloo", batch_size=2, image_size=32, steps=3, warmup_steps=0, num_classes=10,
                     log_every=0, check_replicas_every=1)
    t = Trainer(cfg)
    t.run()                                  # identical replicas: the per-step checks pass
    if not corrupt:
        return "ok"
    if dist.get_rank() == 1:                 # a replica drifts (what a missing stream dependency does)
        with torch.no_grad():
            t.ddp.arena.flat[123] += 1e-3
    try:
        t.ddp.check_replicas()
    except ReplicaDivergence as e:
        return f"caught: {e}"
    return "missed"


@pytest.mark.parametrize("corrupt", [False, True])
def test_replica_divergence_check(corrupt):
    """DataParallel.check_replicas (Trainer check_replicas_every): identical replicas pass every
    step; a parameter that differs on one rank raises ReplicaDivergence on every rank."""
    out = Distributor(num_processes=2, use_gpu=False, timeout_s=300).run(_replicas, corrupt)
    if corrupt:
        assert out.startswith("caught: rank 0"), out
    else:
        assert out == "ok"


def test_adasum_combine_properties():
    """Adasum (Horovod): orthogonal gradients add, identical ones are returned unchanged, and
    scaling one input does not change the other's coefficient's sign / the result's direction."""
    from databricks_distributed_deep_learning_amd.parallel.horovod import adasum_combine, adasum_tree
    a = torch.tensor([1.0, 0.0, 0.0])
    b = torch.tensor([0.0, 2.0, 0.0])
    assert torch.allclose(adasum_combine(a, b), a + b)
    assert torch.allclose(adasum_combine(a, a), a)
    c = torch.tensor([3.0, 1.0, -2.0])
    d = torch.tensor([1.0, -1.0, 0.5])
    ref = (1 - c @ d / (2 * c @ c)) * c + (1 - c @ d / (2 * d @ d)) * d
    assert torch.allclose(adasum_combine(c, d), ref, atol=1e-6)
    # a zero gradient leaves the other one unchanged
    assert torch.allclose(adasum_combine(torch.zeros(3), d), d)
    # tree order: ((0,1),(2,3)); an odd rank is carried up a level
    p = [torch.randn(5, generator=torch.Generator().manual_seed(i)) for i in range(3)]
    assert torch.allclose(adasum_tree(p), adasum_combine(adasum_combine(p[0], p[1]), p[2]))


def _hvd_adasum():
    from databricks_distributed_deep_learning_amd.parallel import hvd
    from databricks_distributed_deep_learning_amd.parallel.horovod import adasum_combine
    hvd.init()
    r = hvd.rank()
    g = [torch.randn(7, generator=torch.Generator().manual_seed(40 + k)) for k in range(2)]
    red = hvd.allreduce(g[r], op=hvd.Adasum)
    err_t = (red - adasum_combine(g[0], g[1])).abs().max().item()
    # DistributedOptimizer(op=Adasum): local step, per-tensor Adasum of the parameter deltas;
    # plain SGD: delta = -lr * g, so p = p0 - lr * Adasum(g0, g1) (Adasum is scale invariant)
    torch.manual_seed(3)
    m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 2))
    x = torch.randn(8, 6, generator=torch.Generator().manual_seed(9))
    grads = []
    for k in range(2):
        m.zero_grad()
        m(x[4 * k:4 * k + 4]).square().sum().backward()
        grads.append([p.grad.clone() for p in m.parameters()])
    opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), named_parameters=m.named_parameters(),
                                   op=hvd.Adasum)
    p0 = [p.detach().clone() for p in m.parameters()]
    opt.zero_grad()
    m(x[4 * r:4 * r + 4]).square().sum().backward()
    opt.step()
    err_o = max((p.detach() - (p0[i] - 0.1 * adasum_combine(grads[0][i], grads[1][i]))).abs().max().item()
                for i, p in enumerate(m.parameters()))
    return err_t, err_o


def _hvd_adasum_tree(n):
    """Recursive-doubling Adasum over n ranks == adasum_tree of the n inputs (incl. an odd
    world: a block without a partner is carried up), identical on every rank."""
    from databricks_distributed_deep_learning_amd.parallel import hvd
    from databricks_distributed_deep_learning_amd.parallel.horovod import adasum_allreduce, adasum_tree
    hvd.init()
    r = hvd.rank()
    g = [torch.randn(11, generator=torch.Generator().manual_seed(70 + k)) for k in range(n)]
    segs = [(0, 4), (4, 7)]
    red = adasum_allreduce(g[r], segs)
    want = torch.cat([adasum_tree([x[o:o + k] for x in g]) for o, k in segs])
    return (red - want).abs().max().item()


@pytest.mark.parametrize("n", [3, 4])
def test_horovod_adasum_recursive_doubling(n):
    res = HorovodRunner(np=n, use_gpu=False).run(_hvd_adasum_tree, n=n)
    assert res < 1e-6, res


def test_horovod_adasum_world2():
    res = HorovodRunner(np=2, use_gpu=False).run(_hvd_adasum)
    assert res[0] < 1e-6 and res[1] < 1e-5, res
