"""Per-module forward divergence native-bf16 vs fp32 reference (GPU debugging aid)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from databricks_distributed_deep_learning_amd import models, ops  # noqa: E402
from databricks_distributed_deep_learning_amd.models.layers import cast_params  # noqa: E402
from databricks_distributed_deep_learning_amd.ops import _native_gemm as NG  # noqa: E402


def capture(model, x, native, force=None):
    outs = {}
    hooks = [m.register_forward_hook(lambda mod, i, o, n=n: outs.__setitem__(n, o.detach().float().clone()))
             for n, m in model.named_modules() if n and isinstance(o := m, torch.nn.Module) and len(list(m.children())) == 0]
    ops.set_native_mode(native)
    with NG.force_kernel(force):
        model(x.to(next(model.parameters()).dtype))
    ops.set_native_mode("auto")
    for h in hooks:
        h.remove()
    return outs


arch = sys.argv[1]
torch.manual_seed(0)
dev = torch.device("cuda")
m = getattr(models, arch)(num_classes=10).to(dev).train()
x = torch.randn(8, 96, 96, 3, device=dev)
ref = capture(copy.deepcopy(m), x, "off")
t16 = capture(cast_params(copy.deepcopy(m), torch.bfloat16), x, "off")
for force in (None, "small", "big", "narrow"):
    nat = capture(cast_params(copy.deepcopy(m), torch.bfloat16), x, "auto", force)
    print("=== force", force)
    for n in ref:
        if n not in nat:
            continue
        e = ((nat[n] - ref[n]).abs().max() / ref[n].abs().max().clamp_min(1e-6)).item()
        et = ((t16[n] - ref[n]).abs().max() / ref[n].abs().max().clamp_min(1e-6)).item()
        flag = "  <<<" if e > 3 * et + 0.02 else ""
        print(f"{n:32s} {tuple(ref[n].shape)!s:22s} native {e:.4f} torch16 {et:.4f}{flag}")
