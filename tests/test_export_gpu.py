"""Native inference graph (BN folded, fused epilogues, hipGraph replay) on the GPU."""
import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu


def test_folded_resnet50_native_and_hipgraph():
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd import ops
    from databricks_distributed_deep_learning_amd.export import FoldedResNet, GraphRunner
    from databricks_distributed_deep_learning_amd.models import resnet50
    torch.manual_seed(0)
    m = resnet50().eval().to(dev)
    x = torch.randn(4, 224, 224, 3, device=dev)
    ops.set_native_mode("off")
    with torch.no_grad():
        ref = m(x)
    ops.set_native_mode("auto")
    f = FoldedResNet(m).to(dev)
    with torch.no_grad():
        y = f(x.to(torch.bfloat16)).float()
    rel = ((y - ref).abs().max() / ref.abs().max()).item()
    assert rel < 5e-2, rel
    g = GraphRunner(f, x.to(torch.bfloat16))
    y2 = g.run(x.to(torch.bfloat16)).float()
    torch.testing.assert_close(y2, y)


def test_bench_runtimes_gpu(tmp_path):
    dev = gpu_device()
    from databricks_distributed_deep_learning_amd.export import bench_runtimes
    from databricks_distributed_deep_learning_amd.models import resnet50
    torch.manual_seed(0)
    rep = bench_runtimes(resnet50(), torch.randn(1, 224, 224, 3, device=dev), iters=5, warmup=2,
                         workdir=str(tmp_path))
    rt = rep["runtimes"]
    assert "native_bf16_folded_hipgraph" in rt
    print({k: round(v["ms"], 3) for k, v in rt.items()})
    oracle = rt["pytorch_eager_fp32"]
    # fp32 graph runtimes: the reference's allclose gate (cv/onnx:144, rtol 1e-5 / atol 1e-4)
    for name in ("torchscript_fp32", "torch_export_fp32"):
        assert rt[name]["allclose_ref_tol"] and rt[name]["top1_agrees"], (name, rt[name])
    # bf16 native runtimes: within bf16 error of the fp32 oracle, and the same top-1 whenever
    # the oracle's top-1 / top-2 margin exceeds that error
    for name in ("native_bf16_eager", "native_bf16_folded", "native_bf16_folded_hipgraph"):
        r = rt[name]
        assert r["max_abs_err"] / oracle["logit_absmax"] < 5e-2, (name, r, oracle)
        if oracle["top12_margin"] > 2 * r["max_abs_err"]:
            assert r["top1_agrees"], (name, r, oracle)
    # the replayed graph is the folded model, bit for bit
    assert rt["native_bf16_folded_hipgraph"]["max_abs_err"] == rt["native_bf16_folded"]["max_abs_err"]
