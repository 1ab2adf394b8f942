"""The notebooks' GPU branch and the TorchDistributor-style launcher on the GPU.

The CPU notebook smoke (tests/test_export_notebooks_cpu.py) hides the GPU, so every
notebook there takes its gloo branch; here the ResNet notebook runs its GPU branch
(RCCL process group, native kernels, ``Distributor(device_count, use_gpu=True)`` --
in-process at one GPU), and ``Distributor(1, use_gpu=True).run(train, cfg)`` is
called directly the way a notebook cell would.
"""
import os
import subprocess
import sys

import pytest

from conftest import gpu_device

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_resnet_notebook_gpu_branch():
    gpu_device()
    env = dict(os.environ, DDL_NOTEBOOK_SMOKE="gpu", PYTHONPATH=ROOT)
    # a fresh notebook process: no rendezvous variables left over from this pytest process
    for k in ("MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "notebooks/cv/resnet_distributed_training.py")],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "'world_size': 1" in r.stdout and "'native': 'auto'" in r.stdout, r.stdout[-2000:]


def test_distributor_train_on_gpu():
    gpu_device()
    from databricks_distributed_deep_learning_amd.config import TrainConfig
    from databricks_distributed_deep_learning_amd.ops import _lib
    from databricks_distributed_deep_learning_amd.parallel import Distributor
    from databricks_distributed_deep_learning_amd.training import train
    cfg = TrainConfig(model="bert_tiny", batch_size=8, seq_len=64, num_classes=2, optimizer="adamw", lr=1e-3,
                      steps=3, warmup_steps=1, log_every=1, pad_fraction=0.25)
    import torch.distributed as dist
    from databricks_distributed_deep_learning_amd.parallel import dist as ddist
    had_pg = dist.is_initialized()
    try:
        s = Distributor(1, use_gpu=True).run(train, cfg)
    finally:
        if not had_pg:
            ddist.destroy()          # later modules bring up their own process group
    assert _lib.available()
    assert s["world_size"] == 1 and s["native"] == "auto" and s["final_loss"] == s["final_loss"]
    assert {"fwd_ms", "bwd_ms", "opt_ms", "comm_wait_ms"} <= set(s["phases_ms"]), s
