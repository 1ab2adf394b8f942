"""Native SyncBatchNorm at world size 2 on one GPU (both ranks on cuda:0, statistics
summed over a gloo group, which reduces CUDA tensors through the host).

Checks the split native path against the CPU reference per rank: dx, and dgamma /
dbeta as THIS rank's partials (the data-parallel reducer sums them across ranks
afterwards, so a kernel that wrote the group-summed row would be `world` times too
large after the reduction).  No ReLU: outputs within bf16 rounding of zero would flip
the mask between the bf16 and fp32 runs (the mask path is covered at world size 1 in
test_comm_gpu.py).  Two backward variants: the BN's own partial pass
(elementwise consumer) and the reduction in the consuming conv's dgrad epilogue."""
import os

import pytest
import torch

from conftest import gpu_device

pytestmark = pytest.mark.gpu


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from databricks_distributed_deep_learning_amd import ops
        from databricks_distributed_deep_learning_amd.ops.conv import conv2d_reference
        from databricks_distributed_deep_learning_amd.ops.norm import sync_batch_norm_reference
        dev = torch.device("cuda", 0)
        C, K = 64, 64
        g = torch.Generator().manual_seed(21)
        x_all = torch.randn(2 * world, 10, 10, C, generator=g) * 1.5 + 0.3
        dy_all = torch.randn(2 * world, 10, 10, K, generator=g)
        gamma0 = torch.rand(C, generator=g) + 0.5
        beta0 = torch.randn(C, generator=g) * 0.1
        w2 = torch.randn(K, 3, 3, C, generator=g) * 0.05
        x, dy = x_all[2 * rank:2 * rank + 2], dy_all[2 * rank:2 * rank + 2]
        # the reference sees the bf16-rounded operands the native path computes on
        x, dy, gamma0, beta0, w2 = (t.to(torch.bfloat16).float() for t in (x, dy, gamma0, beta0, w2))
        errs = {}
        for consumer in ("elementwise", "conv"):
            # reference: fp32 on the CPU, the same gloo group
            xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gamma0, beta0))
            yr = sync_batch_norm_reference(xr, gr, br, torch.zeros(C), torch.ones(C), 0.1, 1e-5, False, None,
                                           dist.group.WORLD)
            zr = conv2d_reference(yr, w2, 1, 1) if consumer == "conv" else yr
            (zr * (dy if consumer == "conv" else dy[..., :C])).sum().backward()
            # native: bf16 on the GPU
            xn = x.to(dev, torch.bfloat16).requires_grad_(True)
            gn = gamma0.to(dev, torch.bfloat16).requires_grad_(True)
            bn = beta0.to(dev, torch.bfloat16).requires_grad_(True)
            yn = ops.batch_norm(xn, gn, bn, torch.zeros(C, device=dev), torch.ones(C, device=dev), True, 0.1,
                                1e-5, False, None, group=dist.group.WORLD)
            zn = ops.conv2d(yn, w2.to(dev, torch.bfloat16), 1, 1) if consumer == "conv" else yn
            dyn = (dy if consumer == "conv" else dy[..., :C]).to(dev, torch.bfloat16)
            zn.backward(dyn)
            torch.cuda.synchronize()

            def rel(a, b):
                a, b = a.detach().float().cpu(), b.detach().float()
                return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()
            errs[consumer] = {"dx": rel(xn.grad, xr.grad), "dgamma": rel(gn.grad, gr.grad),
                              "dbeta": rel(bn.grad, br.grad)}
        q.put((rank, errs))
    except Exception as e:          # surface the failure in the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sync_batchnorm_native_world2_param_grads_are_local_partials():
    gpu_device()
    import torch.multiprocessing as mp
    from databricks_distributed_deep_learning_amd.parallel.dist import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    out = {}
    try:
        for _ in procs:
            rank, res = q.get(timeout=100)
            out[rank] = res
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
    for rank, res in out.items():
        assert isinstance(res, dict), (rank, res)
        for consumer, errs in res.items():
            assert max(errs.values()) < 3e-2, out
