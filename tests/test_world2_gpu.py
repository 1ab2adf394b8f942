"""Multi-rank data-parallel paths on ONE GPU: two ranks on cuda:0 over a gloo group
(gloo reduces CUDA tensors through the host; RCCL refuses two ranks on one device).

* the eager optimizer (per-bucket updates on a side stream during backward, each waiting
  for its bucket's all-reduce handle) == the post-backward step, parameters AND optimizer
  state, at world size 2 -- the multi-rank ordering a missing stream dependency breaks;
* ZeRO-1 on reduce-scatter (local gradient shards, sharded native optimizer kernels,
  per-bucket all-gathers waited by forward pre-hooks) == replicated data parallelism;
* every arm checks after every step that both ranks hold identical parameters
  (``DataParallel.check_replicas``).
"""
import os

import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu


def _rank_main(rank, world, port, q, what):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from databricks_distributed_deep_learning_amd.config import get_preset
        from databricks_distributed_deep_learning_amd.training.loop import Trainer
        finals = []
        arms = (dict(eager_optimizer=True), dict(eager_optimizer=False)) if what == "eager" else \
            (dict(zero_optimizer=True), dict(zero_optimizer=False))
        for arm in arms:
            cfg = get_preset("bert_base_ddp", batch_size=4, seq_len=64, steps=3, warmup_steps=0, log_every=0,
                             backend="gloo", optimizer="adamw", lr=1e-3, bucket_mb=8.0, first_bucket_mb=2.0,
                             check_replicas_every=1, **arm)   # replicas identical after every step
            t = Trainer(cfg)
            if what == "eager":
                assert t.eager_optimizer == arm["eager_optimizer"]
            else:
                assert (t.opt.shard is not None) == arm["zero_optimizer"]
            t.run()
            torch.cuda.synchronize()
            st = {"flat": t.arena.flat.float().clone()}
            if what == "eager":
                st.update({k: v.float().clone() for k, v in t.opt._state_tensors().items()})
            finals.append(st)
            del t
        # (a ZeRO arena is padded to world * 64 elements: compare the common prefix)
        errs = {}
        for k in finals[0]:
            n = min(finals[0][k].numel(), finals[1][k].numel())
            errs[k] = (finals[0][k][:n] - finals[1][k][:n]).abs().max().item()
        q.put((rank, errs))
    except Exception as e:          # surface the failure in the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("what", ["eager", "zero"])
def test_world2_on_one_gpu(what):
    gpu_device()
    import torch.multiprocessing as mp
    from databricks_distributed_deep_learning_amd.parallel.dist import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q, what)) for r in range(2)]
    for pr in procs:
        pr.start()
    out = {}
    try:
        for _ in procs:
            rank, res = q.get(timeout=150)
            out[rank] = res
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
    for rank, res in out.items():
        assert isinstance(res, dict), (rank, res)
        # eager vs post-backward: the same kernels on the same numbers in a different order
        # of launch only; ZeRO: bf16 reduce-scatter vs all-reduce summation order
        tol = 1e-6 if what == "eager" else 2e-2
        assert max(res.values()) <= tol, out
