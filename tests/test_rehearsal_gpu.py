"""The N > 1 step form rehearsed on one GPU.

``dp_rehearsal=True`` at world 1 runs what a data-parallel rank runs -- the native RCCL engine
(``csrc/runtime/comm.cpp``), per-bucket all-reduces overlapped with backward, and the per-bucket
range optimizer started as each bucket's all-reduce completes (``Trainer.overlap_optimizer``) --
instead of the plain world-1 step (one optimizer call over the whole arena, no communicator).
At world 1 an all-reduce is the identity, so both step forms must leave the SAME parameters and
optimizer state: bit for bit, since the range optimizer runs the same elementwise kernel over the
same elements.  The GEMM plan is shared (same process: the second trainer reuses the first one's
tuned kernels), so both runs execute the same kernels in the same order.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(preset, rehearsal, **kw):
    from databricks_distributed_deep_learning_amd.config import get_preset
    from databricks_distributed_deep_learning_amd.training.loop import Trainer
    cfg = get_preset(preset, **kw).replace(steps=3, warmup_steps=0, log_every=0, dp_rehearsal=rehearsal,
                                           phase_timing=True, bucket_mb=8.0, first_bucket_mb=2.0)
    tr = Trainer(cfg)
    out = tr.run()
    flat = tr.arena.flat.detach().clone()
    opt = tr.opt
    state = {k: getattr(opt, k).detach().clone() for k in ("master", "buf", "m", "v") if
             isinstance(getattr(opt, k, None), torch.Tensor) and getattr(opt, k).numel()}
    info = {"comm": tr.ddp.comm, "overlap": tr.overlap_optimizer, "rehearsal": tr.rehearsal,
            "buckets": len(tr.ddp.bucket_sizes_mb())}
    tr.close()
    return out, flat, state, info


@pytest.fixture(scope="module")
def rccl_pg():
    """A 1-rank RCCL process group for this module (what the Trainer would create), torn down at
    the end so later modules can bring up their own."""
    if not torch.cuda.is_available():
        pytest.skip("GPU")
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.parallel import dist as ddist
    mine = not dist.is_initialized()
    ddist.init("auto")
    yield
    if mine and dist.is_initialized():
        dist.destroy_process_group()


@pytest.mark.parametrize("preset,kw", [("resnet50_ddp", dict(batch_size=16)),
                                       ("bert_base_ddp", dict(batch_size=8, dropout=0.1))])
def test_rehearsal_matches_plain_world1_step(rccl_pg, preset, kw):
    from databricks_distributed_deep_learning_amd.parallel.comm import native_available
    if not native_available():
        pytest.skip("RCCL engine unavailable")
    plain, p_flat, p_state, p_info = _run(preset, False, **kw)
    reh, r_flat, r_state, r_info = _run(preset, True, **kw)
    assert not p_info["rehearsal"] and not p_info["overlap"]
    assert r_info["rehearsal"] and r_info["overlap"] and r_info["comm"] == "native" and r_info["buckets"] > 2
    assert reh.get("dp_rehearsal") and reh["rccl"]["nranks"] == 1
    assert "comm_wait+opt_ms" in reh["phases_ms"] and "opt_ms" in plain["phases_ms"]
    assert reh["comm_buckets"], "per-bucket ring timings of the last step"
    assert torch.equal(p_flat, r_flat), (p_flat.float() - r_flat.float()).abs().max()
    assert p_state.keys() == r_state.keys() and p_state
    for k in p_state:
        assert torch.equal(p_state[k], r_state[k]), k
    assert plain["final_loss"] == reh["final_loss"]
