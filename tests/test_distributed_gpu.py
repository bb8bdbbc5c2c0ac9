"""Data parallelism through the GPU training path: 2 ranks on one MI355X (gloo backend).

The node's 8-GPU RCCL run is the driver's; this exercises everything around the collective on a real HIP
stream: the fused blocks writing weight gradients into the flat buffer, gradient-ready notifications, bucketed
all-reduces launched mid-backward (in the gradient dtype, or through an fp32 staging buffer: ``comm = "fp32"``),
the wait before the optimizer.  Both ranks must end with identical gradients and weights, and the all-reduced
gradient must match one process that trains on the concatenated batch (bf16 tolerance).
"""

from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.dist]

CFG = dict(vocab_size=512, context_length=256, d_model=256, num_layers=2, num_heads=4, d_ff=512)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(dev):
    from bpe_transformer.models import TransformerLM

    torch.manual_seed(0)
    return TransformerLM(**CFG, device=dev, dtype=torch.bfloat16)


def _batch(rank: int, dev):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randint(0, CFG["vocab_size"], (2, CFG["context_length"]), generator=g)
    return x.to(dev), torch.roll(x, -1, 1).to(dev)


def _worker(rank, world, port, bucket_mb, comm, out_q, fp8=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")  # both ranks share cuda:0
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed("cuda", backend="gloo")
    model = _model(info.device)
    if fp8:  # fp8 projections incl. the fp8 weight gradients accumulated into the flat buffer's bucket views
        model.enable_fp8()
    eng = TrainEngine(model, info, lr=1e-3, weight_decay=0.0, max_grad_norm=1.0, bucket_mb=bucket_mb,
                      ddp_check_every=1,  # also asserts bit-identical grads / weights across the ranks
                      comm_dtype=torch.float32 if comm == "fp32" else None)
    eng.train_step([_batch(rank, info.device)])
    g1 = eng.flat.grad.float().cpu()
    eng.train_step([_batch(rank, info.device)])
    torch.cuda.synchronize()
    # numpy copies travel by value; torch tensors go through fd sharing whose listener dies with this process
    out_q.put((rank, g1.numpy().copy(), eng.flat.data.float().cpu().numpy().copy(), len(eng.ddp.buckets)))
    cleanup()


def test_dp2_gpu_fp8(gpu_device):
    """Two ranks with fp8 projections (e4m3 forward, e5m2 input and weight gradients, the latter accumulated by the
    split-K fp8 kernel straight into the flat buffer's views): several buckets, gradients and weights identical on
    both ranks after two steps, all finite."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 0.25, "grad", q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (torch.from_numpy(g), torch.from_numpy(d), nb) for r, g, d, nb in (q.get(timeout=240) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][2] > 1
    assert torch.equal(res[0][0], res[1][0]), "all-reduced gradients differ between ranks"
    assert torch.equal(res[0][1], res[1][1]), "ranks diverged"
    assert bool(torch.isfinite(res[0][0]).all()) and float(res[0][0].norm()) > 0


@pytest.mark.parametrize("comm", ["grad", "fp32"])
@pytest.mark.parametrize("bucket_mb", [0.25, 64.0])
def test_dp2_gpu(gpu_device, bucket_mb, comm):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, comm, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (torch.from_numpy(g), torch.from_numpy(d), nb) for r, g, d, nb in (q.get(timeout=240) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if bucket_mb < 1:
        assert res[0][2] > 1, "expected several buckets"
    assert torch.equal(res[0][0], res[1][0]), "all-reduced gradients differ between ranks"
    assert torch.equal(res[0][1], res[1][1]), "ranks diverged"
    # single process on both ranks' sequences: its mean-loss gradient is the DP average
    from bpe_transformer.train.engine import TrainEngine

    eng = TrainEngine(_model(gpu_device), lr=1e-3, weight_decay=0.0, max_grad_norm=1.0)
    x0, y0 = _batch(0, gpu_device)
    x1, y1 = _batch(1, gpu_device)
    eng.train_step([(torch.cat([x0, x1]), torch.cat([y0, y1]))])
    ref = eng.flat.grad.float().cpu()
    err = float((res[0][0] - ref).norm() / ref.norm())
    assert err < 2e-2, err


def _zero_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed("cuda", backend="gloo")
    out = []
    for zero in (0, 1):
        eng = TrainEngine(_model(info.device), info, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0, bucket_mb=0.25,
                          zero=zero, ddp_check_every=1 - zero)  # zero: the forward's fences alone must wait
        for _ in range(2):
            eng.train_step([_batch(rank, info.device)])
        eng.sync_params()
        torch.cuda.synchronize()
        out.append((eng.flat.data.float().cpu().numpy().copy(), float(eng.last_grad_norm), len(eng.ddp.buckets)))
        eng.ddp.remove_hooks()
    out_q.put((rank, out))
    cleanup()


def test_zero1_gpu(gpu_device):
    """Sharded DP (parallel/zero.py) on the GPU path: fused blocks notify gradient readiness, buckets are
    reduced, AdamW runs on each rank's pieces only and the weight all-gathers are waited per module by the next
    forward; the ranks end identical and equal to the unsharded engine (bf16 tolerance)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_zero_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (d0, n0, _), (z0, nz, nb) = res[0]
    d0, z0 = torch.from_numpy(d0), torch.from_numpy(z0)
    assert nb > 2
    assert (res[0][1][0] == res[1][1][0]).all(), "sharded ranks diverged"
    assert abs(n0 - nz) <= 1e-3 * n0
    m = min(d0.numel(), z0.numel())
    err = float((z0[:m] - d0[:m]).abs().max())
    assert err < 2e-2, err
    assert float((z0[:m] != d0[:m]).float().mean()) < 0.01


def _nccl_zero_worker(port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from bpe_transformer.parallel.dist import DistInfo
    from bpe_transformer.train.engine import TrainEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    info = DistInfo(0, 1, 0, dev, "nccl")
    out = []
    for zero in (0, 1):
        eng = TrainEngine(_model(dev), info if zero else None, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0,
                          bucket_mb=0.25, zero=zero)
        for _ in range(2):
            eng.train_step([_batch(0, dev)])
        eng.sync_params()
        torch.cuda.synchronize()
        out.append((eng.flat.data.float().cpu().numpy().copy(), float(eng.last_grad_norm),
                    len(eng.ddp.buckets) if eng.ddp is not None else 0))
    dist.destroy_process_group()
    out_q.put(out)


def test_zero1_rccl_calls_one_rank(gpu_device):
    """The RCCL side of sharded DP on one GPU (a one-rank nccl group): the in-place reduce_scatter_tensor /
    all_gather_into_tensor on flat-buffer views and the scalar norm all-reduce are accepted by the backend and
    the engine trains exactly like the single-process one (the 8-GPU data movement is the driver's run)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_zero_worker, args=(_free_port(), q))
    p.start()
    (d0, n0, _), (z0, nz, nb) = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert nb > 2
    assert abs(n0 - nz) <= 1e-3 * n0
    m = min(d0.shape[0], z0.shape[0])
    d0, z0 = torch.from_numpy(d0[:m]), torch.from_numpy(z0[:m])
    assert float((z0 - d0).abs().max()) < 2e-2
    assert float((z0 != d0).float().mean()) < 0.01
