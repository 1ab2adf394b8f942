"""Export + inference runtime comparison (reference parity).

The reference notebook (``notebooks/cv/onnx_experiments.py``) exports ResNet-50
to ONNX (:33-42), runs it with ONNX Runtime (:77-104) and OpenVINO (:120-140),
runs PyTorch eager (:159-184), checks ORT/OpenVINO parity with
``np.allclose(rtol=1e-5, atol=1e-4)`` (:144), pickles the module (:198), traces
TorchScript (:209-215) and lists artifact sizes (:194,202,219).

MI355X-native equivalent:
  * exporters: TorchScript trace, ``torch.export`` program, safetensors weights,
    a weights_only-loadable state dict, and ONNX when the ``onnx`` package exists
    (it is not installed in this image: reported as skipped, never faked);
  * runtimes: PyTorch eager fp32 (the oracle), TorchScript, our native bf16
    kernels, and our native *inference graph*: BatchNorm folded into the conv
    weights, conv + bias + residual + ReLU fused in the GEMM epilogue, the whole
    forward captured once in a hipGraph and replayed;
  * the same top-5 printout, an allclose parity gate (fp32 backends at the
    reference's tolerances; bf16 backends by top-1/top-5 agreement and max
    error), latency with warm-up + device sync (the reference times one
    unsynchronised sample), and an artifact-size table.
"""
from __future__ import annotations

import copy
import os
import time
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from .. import ops
from ..models.resnet import ResNet


# ------------------------------------------------------------ BN folding
class FoldedConv(nn.Module):
    def __init__(self, w: torch.Tensor, b: torch.Tensor, stride: int, pad: int, relu: bool):
        super().__init__()
        self.register_buffer("weight", w)
        self.register_buffer("bias", b)
        self.stride, self.pad, self.relu = stride, pad, relu

    def forward(self, x, residual=None):
        return ops.conv2d_bias_act(x, self.weight, self.bias, self.stride, self.pad, self.relu, residual)


def _fold(conv, bn, relu: bool, dtype) -> FoldedConv:
    inv = torch.rsqrt(bn.running_var.float() + bn.eps)
    g = bn.weight.float() * inv
    w = conv.weight.float() * g.view(-1, 1, 1, 1)
    b = bn.bias.float() - bn.running_mean.float() * g
    return FoldedConv(w.to(dtype), b.to(dtype), conv.stride, conv.padding, relu)


class FoldedBlock(nn.Module):
    def __init__(self, blk, dtype):
        super().__init__()
        self.bottleneck = hasattr(blk, "conv3")
        self.c1 = _fold(blk.conv1, blk.bn1, True, dtype)
        self.c2 = _fold(blk.conv2, blk.bn2, True, dtype) if self.bottleneck else _fold(blk.conv2, blk.bn2, True, dtype)
        self.c3 = _fold(blk.conv3, blk.bn3, True, dtype) if self.bottleneck else None
        self.down = None
        if blk.downsample is not None:
            self.down = _fold(blk.downsample._modules["0"], blk.downsample._modules["1"], False, dtype)

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        if self.bottleneck:
            return self.c3(self.c2(self.c1(x)), residual=idt)
        return self.c2(self.c1(x), residual=idt)


class FoldedResNet(nn.Module):
    """Inference ResNet: every conv+BN(+add)(+ReLU) is ONE fused GEMM launch."""

    def __init__(self, model: ResNet, dtype=torch.bfloat16):
        super().__init__()
        m = model.eval()
        self.stem = _fold(m.conv1, m.bn1, True, dtype)
        self.blocks = nn.ModuleList([FoldedBlock(b, dtype) for layer in (m.layer1, m.layer2, m.layer3, m.layer4)
                                     for b in layer])
        self.register_buffer("fc_w", m.fc.weight.detach().to(dtype))
        self.register_buffer("fc_b", m.fc.bias.detach().to(dtype))
        self.channels_last_input = m.channels_last_input
        self.dtype = dtype

    @torch.no_grad()
    def forward(self, x):
        if not self.channels_last_input:
            x = x.permute(0, 2, 3, 1).contiguous()
        x = self.stem(x.to(self.dtype))
        x = ops.max_pool2d(x, 3, 2, 1)
        for b in self.blocks:
            x = b(x)
        return ops.linear(ops.global_avg_pool(x), self.fc_w, self.fc_b)


class GraphRunner:
    """Capture ``fn(static_input)`` once into a hipGraph; ``run(x)`` copies x in and replays."""

    def __init__(self, fn, example: torch.Tensor, warmup: int = 3):
        self.fn = fn
        self.static_in = example.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.fn(self.static_in)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_out = self.fn(self.static_in)

    def run(self, x: torch.Tensor) -> torch.Tensor:
        self.static_in.copy_(x)
        self.graph.replay()
        return self.static_out


# ------------------------------------------------------------ exporters
def export_model(model: nn.Module, example: torch.Tensor, fmt: str, path: str) -> Optional[str]:
    """Write ``model`` in ``fmt``; returns the path, or None when the format's
    package is unavailable (onnx)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    model = model.eval()
    if fmt == "torchscript":
        with torch.no_grad():
            torch.jit.trace(model, example).save(path)
    elif fmt == "torch_export":
        ep = torch.export.export(model, (example,))
        torch.export.save(ep, path)
    elif fmt == "safetensors":
        from safetensors.torch import save_file
        save_file({k: v.detach().cpu().contiguous().clone() for k, v in model.state_dict().items()}, path)
    elif fmt == "state_dict":
        torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, path)
    elif fmt == "onnx":
        try:
            import onnx  # noqa: F401
        except ImportError:
            return None
        torch.onnx.export(model, example, path, export_params=True, opset_version=12, do_constant_folding=True,
                          input_names=["input"], output_names=["output"])
    else:
        raise ValueError(fmt)
    return path


def artifact_sizes(paths: Dict[str, Optional[str]]) -> Dict[str, Optional[int]]:
    return {k: (os.path.getsize(p) if p and os.path.exists(p) else None) for k, p in paths.items()}


def load_state_dict_safely(path: str) -> Dict[str, torch.Tensor]:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


# ------------------------------------------------------------ runtime comparison
def _timed(fn, x, iters: int, warmup: int, device) -> (torch.Tensor, float):
    out = None
    for _ in range(warmup):
        out = fn(x)
    if device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        out = fn(x)
    if device.type == "cuda":
        torch.cuda.synchronize()
    return out, (time.perf_counter() - t0) * 1000.0 / iters


def top5(logits: torch.Tensor, categories: Optional[List[str]] = None):
    p, v, i = ops.softmax_topk(logits.float().cpu(), 5)
    names = categories or [f"class_{k}" for k in range(logits.shape[-1])]
    return [(names[int(k)], float(s)) for k, s in zip(i[0], v[0])]


def _ort_session(path: Optional[str]):
    """ONNX Runtime CPU session of ``path``; None when onnx / onnxruntime are not installed."""
    if path is None:
        return None
    try:
        import onnxruntime
    except ImportError:
        return None
    return onnxruntime.InferenceSession(path, providers=["CPUExecutionProvider"])


def bench_runtimes(model: ResNet, x: torch.Tensor, iters: int = 50, warmup: int = 5,
                   categories: Optional[List[str]] = None, workdir: str = "/tmp/ddl_export",
                   rtol: float = 1e-5, atol: float = 1e-4) -> Dict[str, object]:
    """Run every available backend on ``x`` (NHWC batch) and compare with eager fp32."""
    device = x.device
    model = model.eval()
    results: Dict[str, Dict[str, object]] = {}
    prev_mode = ops.native_mode()
    # oracle: PyTorch eager fp32 (stock ops, reference math)
    ops.set_native_mode("off")
    ref_model = copy.deepcopy(model).float().to(device)
    with torch.no_grad():
        ref, ms = _timed(ref_model, x.float(), iters, warmup, device)
    t2 = ref.float().topk(2, dim=-1).values
    results["pytorch_eager_fp32"] = {"ms": ms, "top5": top5(ref, categories),
                                     "logit_absmax": float(ref.float().abs().max()),
                                     "top12_margin": float((t2[..., 0] - t2[..., 1]).min())}
    # TorchScript trace of the fp32 model
    ts_path = os.path.join(workdir, "traced_resnet_model.pt")
    export_model(ref_model, x.float(), "torchscript", ts_path)
    ts = torch.jit.load(ts_path, map_location=device)
    with torch.no_grad():
        out, ms = _timed(ts, x.float(), iters, warmup, device)
    results["torchscript_fp32"] = {"ms": ms, "out": out}
    # torch.export program of the same fp32 model (the ahead-of-time graph path)
    ep_path = export_model(ref_model, x.float(), "torch_export", os.path.join(workdir, "resnet.pt2"))
    ep = torch.export.load(ep_path).module()
    with torch.no_grad():
        out, ms = _timed(ep, x.float(), iters, warmup, device)
    results["torch_export_fp32"] = {"ms": ms, "out": out}
    # ONNX Runtime CPU EP, as the reference's session (cv/onnx:77-83, 91-101), when installed
    onnx_path = export_model(copy.deepcopy(ref_model).cpu(), x.float().cpu(), "onnx",
                             os.path.join(workdir, "resnet50.onnx"))
    sess = _ort_session(onnx_path)
    if sess is not None:
        out, ms = _timed(lambda a: torch.from_numpy(sess.run([], {"input": a.cpu().numpy()})[0]).to(device),
                         x.float(), iters, warmup, device)
        results["onnxruntime_cpu_fp32"] = {"ms": ms, "out": out}
    ops.set_native_mode(prev_mode)
    if device.type == "cuda" and ops.native_available():
        nat = copy.deepcopy(model).to(device)
        from ..models import cast_params
        cast_params(nat, torch.bfloat16)
        with torch.no_grad():
            out, ms = _timed(nat, x.to(torch.bfloat16), iters, warmup, device)
        results["native_bf16_eager"] = {"ms": ms, "out": out}
        folded = FoldedResNet(model.to(device)).to(device)
        with torch.no_grad():
            out, ms = _timed(folded, x.to(torch.bfloat16), iters, warmup, device)
        results["native_bf16_folded"] = {"ms": ms, "out": out}
        g = GraphRunner(folded, x.to(torch.bfloat16))
        out, ms = _timed(g.run, x.to(torch.bfloat16), iters, warmup, device)
        results["native_bf16_folded_hipgraph"] = {"ms": ms, "out": out.clone()}
    # parity vs the fp32 oracle
    for name, r in results.items():
        if "out" not in r:
            continue
        o = r.pop("out").float()
        r["max_abs_err"] = float((o - ref.float()).abs().max())
        r["allclose_ref_tol"] = bool(torch.allclose(o, ref.float(), rtol=rtol, atol=atol))
        r["top1_agrees"] = bool((o.argmax(-1) == ref.argmax(-1)).all())
        r["top5"] = top5(o, categories)
    # artifacts
    paths = {
        "torchscript": ts_path,
        "safetensors": export_model(model.cpu().float(), x.float().cpu(), "safetensors",
                                    os.path.join(workdir, "model.safetensors")),
        "state_dict": export_model(model.cpu().float(), x.float().cpu(), "state_dict",
                                   os.path.join(workdir, "model_state.pt")),
        "onnx": onnx_path,
        "torch_export": ep_path,
    }
    return {"runtimes": results, "artifact_bytes": artifact_sizes(paths)}
