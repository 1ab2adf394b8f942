"""Reference-parity export/inference harness and notebooks, on CPU."""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_export_formats_roundtrip(tmp_path):
    from databricks_distributed_deep_learning_amd.export import export_model, load_state_dict_safely, artifact_sizes
    from databricks_distributed_deep_learning_amd.models import resnet18
    torch.manual_seed(0)
    m = resnet18(num_classes=10).eval()
    x = torch.randn(1, 32, 32, 3)
    paths = {}
    for fmt, name in [("torchscript", "m.pt"), ("safetensors", "m.safetensors"), ("state_dict", "sd.pt"),
                      ("torch_export", "m.pt2"), ("onnx", "m.onnx")]:
        paths[fmt] = export_model(m, x, fmt, str(tmp_path / name))
    sizes = artifact_sizes(paths)
    assert sizes["torchscript"] > 0 and sizes["safetensors"] > 0 and sizes["state_dict"] > 0
    with torch.no_grad():
        ref = m(x)
        ts = torch.jit.load(paths["torchscript"])
        torch.testing.assert_close(ts(x), ref, rtol=1e-5, atol=1e-4)   # reference notebook's tolerance
        ep = torch.export.load(paths["torch_export"])
        torch.testing.assert_close(ep.module()(x), ref, rtol=1e-5, atol=1e-4)
    for key in ("safetensors", "state_dict"):
        m2 = resnet18(num_classes=10).eval()
        m2.load_state_dict(load_state_dict_safely(paths[key]))
        with torch.no_grad():
            torch.testing.assert_close(m2(x), ref)


def test_folded_resnet_matches_eval_model_cpu():
    from databricks_distributed_deep_learning_amd.export import FoldedResNet
    from databricks_distributed_deep_learning_amd.models import resnet50
    torch.manual_seed(0)
    m = resnet50(num_classes=10).eval()
    for mod in m.modules():
        if hasattr(mod, "running_mean"):
            mod.running_mean.uniform_(-0.2, 0.2)
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.data.uniform_(0.5, 1.5)
    x = torch.randn(2, 64, 64, 3)
    f = FoldedResNet(m, dtype=torch.float32)
    with torch.no_grad():
        torch.testing.assert_close(f(x), m(x), rtol=1e-4, atol=1e-4)


def _has(mod):
    try:
        __import__(mod)
        return True
    except ImportError:
        return False


def test_bench_runtimes_cpu(tmp_path):
    from databricks_distributed_deep_learning_amd.export import bench_runtimes
    from databricks_distributed_deep_learning_amd.models import resnet18
    torch.manual_seed(0)
    rep = bench_runtimes(resnet18(num_classes=10), torch.randn(1, 32, 32, 3), iters=1, warmup=1,
                         workdir=str(tmp_path))
    rt = rep["runtimes"]
    for name in ("torchscript_fp32", "torch_export_fp32"):
        assert rt[name]["allclose_ref_tol"] and rt[name]["top1_agrees"], name
    # ONNX Runtime runs only where onnx + onnxruntime are installed (neither is in this image)
    assert ("onnxruntime_cpu_fp32" in rt) == (rep["artifact_bytes"]["onnx"] is not None and _has("onnxruntime"))
    assert len(rt["pytorch_eager_fp32"]["top5"]) == 5
    assert rep["artifact_bytes"]["onnx"] is None or rep["artifact_bytes"]["onnx"] > 0


@pytest.mark.parametrize("nb", ["notebooks/cv/onnx_experiments.py", "notebooks/cv/resnet_distributed_training.py",
                                "notebooks/nlp/bert_finetune_distributed.py", "notebooks/nlp/bert_large_lamb.py",
                                "notebooks/cv/vit_training.py"])
def test_notebook_smoke(nb):
    src = open(os.path.join(ROOT, nb)).read()
    assert src.startswith("# Databricks notebook source")
    assert "# COMMAND ----------" in src
    env = dict(os.environ, DDL_NOTEBOOK_SMOKE="1", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, nb)], env=env, capture_output=True, text=True,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
