"""Single-node multi-process launcher: TorchDistributor-style API (north-star N1).

``Distributor(num_processes=8, local_mode=True, use_gpu=True).run(train_fn, *args)``
spawns one process per GPU, wires the torchrun environment
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT), pins each child to
its GPU, initialises the process group (RCCL on GPU, gloo on CPU), runs
``train_fn`` and returns rank 0's return value.  The first child failure is
re-raised in the parent with the child's traceback and the surviving siblings
are terminated (failure detection).

``train_fn`` may be defined in a notebook cell or an interactive ``__main__``:
the function and its arguments are serialised by value with ``cloudpickle``
(when importable; plain pickle otherwise) and rebuilt in each child before the
call, the way TorchDistributor ships a notebook-local function to its workers.

If the caller is already inside a torchrun / launcher world (``RANK`` set and
``WORLD_SIZE`` matches) the function runs in-process instead of re-spawning, so
the same notebook ``train()`` works under ``python -m torch.distributed.run``.

Reference context: the reference notebook runs everything in the single
Databricks driver REPL; this is the MI355X replacement for the
HorovodRunner / TorchDistributor entrypoint named in BASELINE.json:5.
"""
from __future__ import annotations

import os
import pickle
import sys
import time
import traceback
from typing import Any, Callable, Dict, Optional

import torch.multiprocessing as mp

from . import dist as ddist


class ChildFailed(RuntimeError):
    def __init__(self, rank: int, exc_type: str, message: str, tb: str):
        super().__init__(f"rank {rank} failed with {exc_type}: {message}\n--- child traceback ---\n{tb}")
        self.rank = rank
        self.exc_type = exc_type
        self.child_traceback = tb


def _dumps(obj) -> bytes:
    """By-value serialisation of a callable + arguments: cloudpickle pickles functions and
    classes defined in ``__main__`` / a notebook cell (plain pickle only references them by
    name, which a spawned child cannot resolve)."""
    try:
        import cloudpickle
    except ImportError:      # pragma: no cover - cloudpickle ships in this image
        return pickle.dumps(obj)
    try:
        return cloudpickle.dumps(obj)
    except Exception as e:  # noqa: BLE001
        # cloudpickle trips over some extension objects a function's code merely names
        # (e.g. a local ``from pkg import ops`` next to a global ``torch``: it drags in
        # ``torch.ops``).  By-reference pickling still works for functions of an
        # importable module or of a script file (spawned children re-import it).
        try:
            return pickle.dumps(obj)
        except Exception:
            raise e from None


def _child_entry(rank: int, world: int, payload: bytes, env: Dict[str, str],
                 result_q, init_pg: bool, backend: str, use_gpu: bool) -> None:
    os.environ.update(env)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_WORLD_SIZE"] = str(world)
    try:
        fn, args, kwargs = pickle.loads(payload)   # cloudpickle output loads with pickle
        if init_pg:
            ddist.init(backend=backend, use_gpu=use_gpu)
        out = fn(*args, **kwargs)
        if rank == 0:
            try:
                pickle.dumps(out)
            except Exception:
                out = repr(out)
            result_q.put(("ok", rank, out))
        else:
            result_q.put(("done", rank, None))
    except BaseException as e:  # noqa: BLE001 - propagate everything to the parent
        result_q.put(("err", rank, (type(e).__name__, str(e), traceback.format_exc())))
    finally:
        try:
            if init_pg:
                ddist.destroy()
        except Exception:
            pass


class Distributor:
    """Run a function on ``num_processes`` local ranks.

    Parameters mirror the public ``pyspark.ml.torch.distributor.TorchDistributor``
    surface (num_processes, local_mode, use_gpu).  ``local_mode=False`` is
    accepted for API compatibility; there is one node, so it behaves the same.
    """

    def __init__(self, num_processes: int = 1, local_mode: bool = True, use_gpu: Optional[bool] = None,
                 backend: str = "auto", init_process_group: bool = True, timeout_s: float = 3600.0,
                 master_port: Optional[int] = None, env: Optional[Dict[str, str]] = None):
        if num_processes < 1:
            raise ValueError("num_processes must be >= 1")
        self.num_processes = num_processes
        self.local_mode = local_mode
        if use_gpu is None:
            import torch
            use_gpu = torch.cuda.device_count() > 0
        self.use_gpu = use_gpu
        if use_gpu:
            import torch
            n = torch.cuda.device_count()
            if n and num_processes > n:
                raise ValueError(f"num_processes={num_processes} > visible GPUs ({n})")
        self.backend = ddist.resolve_backend(backend, use_gpu)
        self.init_process_group = init_process_group
        self.timeout_s = timeout_s
        self.master_port = master_port
        self.extra_env = dict(env or {})

    def _in_existing_world(self) -> bool:
        return ("RANK" in os.environ and "WORLD_SIZE" in os.environ
                and int(os.environ["WORLD_SIZE"]) == self.num_processes
                and os.environ.get("DDL_LAUNCHER_CHILD") != "1" and self.num_processes > 1)

    def run(self, fn: Callable, *args, **kwargs) -> Any:
        if self._in_existing_world():
            if self.init_process_group:
                ddist.init(backend=self.backend, use_gpu=self.use_gpu)
            return fn(*args, **kwargs)
        if self.num_processes == 1:
            # in-notebook path: no spawn, 1-rank group so the same code runs
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("LOCAL_RANK", "0")
            if self.init_process_group:
                ddist.init(backend=self.backend, use_gpu=self.use_gpu)
            return fn(*args, **kwargs)
        env = {
            "MASTER_ADDR": "127.0.0.1",
            "MASTER_PORT": str(self.master_port or ddist.free_port()),
            "HSA_ENABLE_IPC_MODE_LEGACY": "0",
            "DDL_LAUNCHER_CHILD": "1",
        }
        env.update(self.extra_env)
        payload = _dumps((fn, args, kwargs))
        ctx = mp.get_context("spawn")
        q = ctx.SimpleQueue()
        procs = []
        for r in range(self.num_processes):
            p = ctx.Process(target=_child_entry,
                            args=(r, self.num_processes, payload, env, q,
                                  self.init_process_group, self.backend, self.use_gpu),
                            daemon=False)
            p.start()
            procs.append(p)
        return self._supervise(procs, q)

    def _supervise(self, procs, q) -> Any:
        deadline = time.time() + self.timeout_s
        result = None
        finished = set()
        failure: Optional[ChildFailed] = None
        while len(finished) < len(procs):
            while not q.empty():
                kind, rank, payload = q.get()
                finished.add(rank)
                if kind == "ok":
                    result = payload
                elif kind == "err" and failure is None:
                    failure = ChildFailed(rank, *payload)
            if failure is not None:
                break
            dead = [i for i, p in enumerate(procs) if not p.is_alive() and i not in finished]
            if dead:
                time.sleep(0.2)  # let a final queue message land
                if not q.empty():
                    continue
                i = dead[0]
                failure = ChildFailed(i, "ProcessExit", f"exit code {procs[i].exitcode}", "")
                break
            if time.time() > deadline:
                failure = ChildFailed(-1, "Timeout", f"launcher timeout after {self.timeout_s}s", "")
                break
            time.sleep(0.05)
        if failure is not None:
            for p in procs:
                if p.is_alive():
                    p.terminate()
            for p in procs:
                p.join(timeout=10)
                if p.is_alive():
                    p.kill()
            raise failure
        for p in procs:
            p.join(timeout=60)
        return result


TorchDistributor = Distributor


def main(argv=None) -> int:
    """``python -m databricks_distributed_deep_learning_amd.parallel.launcher -n 8 script.py args``.

    A torchrun-compatible CLI: spawns ``-n`` children running ``script.py`` with
    the torchrun environment set.  Children are plain subprocesses started before
    any GPU initialisation in the parent.
    """
    import argparse
    import subprocess
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", "--nproc", type=int, default=1)
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    port = a.master_port or ddist.free_port()
    procs = []
    for r in range(a.nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.nproc),
                   LOCAL_WORLD_SIZE=str(a.nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, a.script] + a.args, env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:
                        q.terminate()
            time.sleep(0.1)
    finally:
        for p in procs:
            p.kill()
    return rc


if __name__ == "__main__":
    sys.exit(main())
