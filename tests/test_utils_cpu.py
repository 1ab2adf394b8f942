"""Observability helpers: JSONL log + optional MLflow mirror."""
import json
import sys
import types


def test_jsonl_logger_and_mlflow_mirror(tmp_path, monkeypatch):
    from databricks_distributed_deep_learning_amd.utils.metrics import JsonlLogger
    calls = []
    fake = types.ModuleType("mlflow")
    fake.log_metrics = lambda metrics, step: calls.append((metrics, step))
    monkeypatch.setitem(sys.modules, "mlflow", fake)
    path = tmp_path / "log" / "train.jsonl"
    lg = JsonlLogger(str(path), mlflow=True)
    lg.log({"step": 3, "loss": 1.5, "samples_per_sec": 100, "model": "resnet18", "ok": True})
    rec = json.loads(path.read_text().splitlines()[0])
    assert rec["loss"] == 1.5 and rec["model"] == "resnet18" and "ts" in rec
    assert calls == [({"loss": 1.5, "samples_per_sec": 100.0}, 3)]


def test_mlflow_off_by_default(tmp_path, monkeypatch):
    from databricks_distributed_deep_learning_amd.utils.metrics import JsonlLogger
    monkeypatch.delenv("DDL_MLFLOW", raising=False)
    lg = JsonlLogger(str(tmp_path / "a.jsonl"))
    assert lg._mlflow is None
    lg.log({"step": 0, "loss": 2.0})
    # a non-main rank (enabled=False) writes nothing and mirrors nothing
    off = JsonlLogger(str(tmp_path / "b.jsonl"), enabled=False, mlflow=True)
    off.log({"step": 0, "loss": 2.0})
    assert not (tmp_path / "b.jsonl").exists() and off._mlflow is None


def test_transposed_weight_cache_follows_flat_optimizer():
    """W^T cached for the NT dgrad is keyed on the arena generation the flat optimizers
    bump (their writes bypass the parameter views' version counters)."""
    import torch
    from databricks_distributed_deep_learning_amd.ops._native_linear import _transposed
    from databricks_distributed_deep_learning_amd.optim import FlatAdamW, FlatSGD, ParamArena
    for cls in (FlatSGD, FlatAdamW):
        torch.manual_seed(0)
        lin = torch.nn.Linear(16, 8)
        arena = ParamArena(list(lin.named_parameters()))
        opt = cls(arena, lr=0.5)
        for _ in range(3):
            assert torch.equal(_transposed(lin.weight, lin.weight), lin.weight.t())
            arena.grad.normal_()
            before = lin.weight.detach().clone()
            opt.step()
            assert not torch.equal(before, lin.weight)
        st = opt.state_dict()
        _transposed(lin.weight, lin.weight)
        arena.grad.normal_()
        opt.step()
        opt.load_state_dict(st)           # weights restored from the master copy
        assert torch.equal(_transposed(lin.weight, lin.weight), lin.weight.t())


def test_phase_timer_pending_is_bounded():
    """Without log points the pending marks are folded once max_pending steps accumulate, and
    the summary still averages over every step."""
    import torch
    from databricks_distributed_deep_learning_amd.utils.metrics import PhaseTimer
    pt = PhaseTimer(torch.device("cpu"), max_pending=4)
    for _ in range(10):
        pt.begin()
        pt.mark("fwd")
        pt.mark("bwd")
        pt.end_step()
        assert len(pt._pending) <= 4
    out = pt.summary(reset=True)
    assert pt.steps == 0 and set(out) == {"fwd_ms", "bwd_ms"}
