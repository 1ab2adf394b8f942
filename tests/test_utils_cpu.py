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
