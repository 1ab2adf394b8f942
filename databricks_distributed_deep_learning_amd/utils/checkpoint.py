"""Checkpoint / resume.

The reference only *saves* — a whole-module pickle (``torch.save(resnet50, ...)``,
``notebooks/cv/onnx_experiments.py:198``) and a TorchScript trace (:215) — with
no optimizer state and no load path.  Here a checkpoint is a directory:

* ``model.safetensors``  - weights (no pickle: loading executes nothing)
* ``optim.safetensors``  - flat optimizer state (fp32 master, moments)
* ``rng.safetensors``    - torch CPU generator state (it draws the dropout seeds,
  ``ops/_native_elementwise.py`` ``new_seed``) and the device generator state
* ``meta.json``          - step, config, optimizer scalars, data-loader position

With the RNG streams and the loader position restored, a resumed run replays
exactly the batches and dropout masks the uninterrupted run would have drawn
(bit-identical on the CPU path; tested in tests/test_distributed_cpu.py).

Every rank gathers the optimizer state (collective when it is sharded), rank 0
writes, every rank barriers, every rank loads (collective C5).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional

import torch

from ..parallel import dist as ddist


def _cpu(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {k: v.detach().to("cpu").contiguous() for k, v in sd.items() if isinstance(v, torch.Tensor)}


def _rng_state() -> Dict[str, torch.Tensor]:
    st = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def _set_rng_state(st: Dict[str, torch.Tensor]) -> None:
    if "cpu" in st:
        torch.set_rng_state(st["cpu"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def save(path: str, model: torch.nn.Module, optimizer=None, step: int = 0, config: Optional[Dict] = None,
         extra: Optional[Dict[str, Any]] = None, loader=None) -> None:
    from safetensors.torch import save_file
    # every rank takes the optimizer state: a sharded (ZeRO-1) optimizer all-gathers its
    # slices inside state_dict(), a collective all ranks must enter in the same order
    st = optimizer.state_dict() if optimizer is not None else None
    if ddist.is_main():
        os.makedirs(path, exist_ok=True)
        msd = model.state_dict()
        # safetensors refuses shared storage; clone so views of the arena are independent
        save_file({k: v.clone() for k, v in _cpu(msd).items()}, os.path.join(path, "model.safetensors"))
        meta: Dict[str, Any] = {"step": step, "config": config or {}, "extra": extra or {}}
        if st is not None:
            tensors = {k: v for k, v in st.items() if isinstance(v, torch.Tensor)}
            scalars = {k: v for k, v in st.items() if not isinstance(v, torch.Tensor)}
            save_file(_cpu(tensors), os.path.join(path, "optim.safetensors"))
            meta["optimizer"] = scalars
        meta["rng"] = {"torch_initial_seed": int(torch.initial_seed())}
        save_file(_rng_state(), os.path.join(path, "rng.safetensors"))
        if loader is not None and hasattr(loader, "state_dict"):
            meta["loader"] = loader.state_dict()
        tmp = os.path.join(path, "meta.json.tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True, default=str)
        os.replace(tmp, os.path.join(path, "meta.json"))
    del st
    ddist.barrier()


def load(path: str, model: torch.nn.Module, optimizer=None, map_location=None, loader=None,
         restore_rng: bool = True) -> Dict[str, Any]:
    from safetensors.torch import load_file
    ddist.barrier()
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    dev = map_location or next(model.parameters()).device
    msd = load_file(os.path.join(path, "model.safetensors"), device="cpu")
    own = model.state_dict()
    with torch.no_grad():
        for k, v in msd.items():
            if k in own:
                own[k].copy_(v.to(own[k].dtype))
    if optimizer is not None and os.path.exists(os.path.join(path, "optim.safetensors")):
        ost = load_file(os.path.join(path, "optim.safetensors"), device="cpu")
        st = dict(meta.get("optimizer", {}))
        st.update({k: v.to(dev) for k, v in ost.items()})
        optimizer.load_state_dict(st)
    if loader is not None and "loader" in meta and hasattr(loader, "load_state_dict"):
        loader.load_state_dict(meta["loader"])
    rng = os.path.join(path, "rng.safetensors")
    if restore_rng and os.path.exists(rng):
        _set_rng_state(load_file(rng, device="cpu"))
    return meta


def latest(path: str) -> Optional[str]:
    return path if os.path.exists(os.path.join(path, "meta.json")) else None
