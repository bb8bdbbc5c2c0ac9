"""Data parallelism at the node's real rank count (8), on the CPU (gloo), plus the gradient / wire dtype options.

The driver's scaling run uses 8 ranks; world-size-dependent logic -- bucket cuts, ZeRO-1's ``world x 64`` padding
and piece ownership, the bench's whole-job numbers -- is exercised here at N = 8, not only at 2 or 3.  Also:
fp32 gradient buffers (``FlatParameters(grad_dtype=fp32)`` with bf16 parameters), an fp32 all-reduce of bf16
gradients (``BucketedAllReduce(comm_dtype=...)``), and resuming a ZeRO-1 checkpoint on another world size.
"""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.dist


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(dtype=torch.float32):
    from bpe_transformer.models import TransformerLM

    torch.manual_seed(0)
    return TransformerLM(200, 32, 32, 2, 2, 64).to(dtype)


def _batch(rank: int, step: int):
    g = torch.Generator().manual_seed(100 + 17 * rank + 1000 * step)
    x = torch.randint(0, 200, (2, 32), generator=g)
    return x, torch.roll(x, -1, 1)


def _spawn(fn, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=fn, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)


def _dp_worker(rank, world, port, zero, out_q):
    _env(rank, world, port)
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed("cpu")
    eng = TrainEngine(_model(), info, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5, bucket_mb=0.01, zero=zero,
                      ddp_check_every=1)
    for step in range(2):
        eng.train_step([_batch(rank, step)])
    eng.sync_params()
    eng.gather_optimizer_state()
    sd = eng.state_dict()
    pieces = list(getattr(eng.ddp, "pieces", []))
    out_q.put((rank, (eng.flat.data.numpy().copy(), sd["exp_avg"].numpy().copy(), len(eng.ddp.buckets), pieces,
                      eng.flat.numel)))
    cleanup()


def test_dp8_matches_single_process():
    """8 ranks, one micro-batch each, tiny buckets: every rank ends identical (the per-step consistency check is
    on) and equal to one process training on the 8 micro-batches concatenated."""
    res = _spawn(_dp_worker, 8, 0)
    for r in range(1, 8):
        assert (res[r][0] == res[0][0]).all(), f"rank {r} diverged"
    assert res[0][2] > 4, "expected many buckets"
    from bpe_transformer.train.engine import TrainEngine

    eng = TrainEngine(_model(), lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    for step in range(2):
        bs = [_batch(r, step) for r in range(8)]
        eng.train_step([(torch.cat([b[0] for b in bs]), torch.cat([b[1] for b in bs]))])
    torch.testing.assert_close(torch.from_numpy(res[0][0]), eng.flat.data, atol=5e-5, rtol=1e-4)


def test_zero1_8ranks_matches_unsharded():
    """ZeRO-1 at world 8: pieces are 64-aligned, disjoint and tile the (world x 64)-padded buffer; weights and
    moments equal the unsharded 8-rank run's."""
    z = _spawn(_dp_worker, 8, 1)
    d = _spawn(_dp_worker, 8, 0)
    for r in range(1, 8):
        assert (z[r][0] == z[0][0]).all() and (z[r][1] == z[0][1]).all(), f"rank {r} differs"
    numel = z[0][4]
    assert numel % (64 * 8) == 0
    cover = torch.zeros(numel, dtype=torch.int32)
    for r in range(8):
        for s, e in z[r][3]:
            assert s % 64 == 0 and e % 64 == 0
            cover[s:e] += 1
    assert bool((cover == 1).all())
    a, b = torch.from_numpy(z[0][0]), torch.from_numpy(d[0][0])
    m = min(a.numel(), b.numel())
    torch.testing.assert_close(a[:m], b[:m], atol=2e-4, rtol=1e-5)
    a, b = torch.from_numpy(z[0][1]), torch.from_numpy(d[0][1])
    torch.testing.assert_close(a, b[: a.numel()], atol=1e-7, rtol=1e-5)


def test_bench_contract_eight_ranks_cpu(tmp_path):
    """bench.py under torch.distributed.run with 8 ranks (gloo): one JSON line from rank 0, dp8, global batch 8x."""
    port = _free_port()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "8", "--device", "cpu", "--model", "tinystories-17m", "--seq", "16", "--batch", "1",
           "--steps", "2", "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 8
    assert out["allreduce_dtype"] == "float32" and out["grad_dtype"] == "float32"  # CPU plumbing config is fp32
    d = out["dist"]
    assert d["world_size"] == 8 and d["backend"] == "gloo" and d["buckets"] == len(d["bucket_mb"]) >= 1
    assert d["consistency_check"] == "grad+data bit-identical across ranks"
    assert abs(out["value"] - 2 * 8 * 16 / (out["ms_per_step"] * 2 / 1000)) < 0.02 * out["value"]


def _comm_worker(rank, world, port, comm, out_q):
    _env(rank, world, port)
    from bpe_transformer.optim.flat import FlatParameters
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.parallel.ddp import BucketedAllReduce

    init_distributed("cpu")
    flat = FlatParameters.from_module(_model(torch.bfloat16))
    ar = BucketedAllReduce(flat, bucket_mb=0.01, overlap=False, comm_dtype=comm)
    g = torch.Generator().manual_seed(7 + rank)
    vals = (1.0 + torch.rand(flat.numel, generator=g) / 64).to(torch.bfloat16)  # many bf16 ulps apart per rank
    flat.grad.copy_(vals)
    ar.start()
    ar.finish()
    out_q.put((rank, (vals.float().numpy(), flat.grad.float().numpy())))
    cleanup()


def test_allreduce_in_fp32_for_bf16_grads():
    """bf16 gradients all-reduced in fp32 (comm_dtype) equal the exact fp32 mean rounded to bf16 once; the
    bf16-wire reduction (gloo sums in bf16 rank by rank) is measurably further from it."""
    world = 4
    r32 = _spawn(_comm_worker, world, torch.float32)
    r16 = _spawn(_comm_worker, world, None)
    vals = torch.stack([torch.from_numpy(r32[r][0]) for r in range(world)]).double()
    exact = (vals.sum(0) / world).float().to(torch.bfloat16).float()
    got32 = torch.from_numpy(r32[0][1])
    got16 = torch.from_numpy(r16[0][1])
    assert torch.equal(got32, exact)
    assert (got16 != exact).float().mean() > 0.01


def test_bf16_wire_error_bound_at_eight_ranks():
    """The default wire dtype decision (docs/performance.md "Streams and data parallelism"): with bf16 gradients
    all-reduced in bf16 at N = 8 (gloo adds rank by rank in bf16, as a ring adds hop by hop), the mean lands within
    2 bf16 ulps of the exact fp32 mean rounded once, and within 1 ulp for most elements -- the size of the rounding
    every bf16 weight gradient already carries -- so bf16 stays the default wire dtype and ``--comm-dtype fp32``
    is the exact option."""
    world = 8
    r16 = _spawn(_comm_worker, world, None)
    vals = torch.stack([torch.from_numpy(r16[r][0]) for r in range(world)]).double()
    exact = (vals.sum(0) / world).float().to(torch.bfloat16).float()
    got16 = torch.from_numpy(r16[0][1])
    ulps = (got16.double() - exact.double()).abs() / 2.0**-7  # every value lies in [1, 2): one bf16 ulp is 2^-7
    for r in range(1, world):  # every rank holds the same result
        assert torch.equal(torch.from_numpy(r16[r][1]), got16)
    assert ulps.max() <= 2.0, float(ulps.max())
    assert (ulps <= 1.0).float().mean() > 0.9, float((ulps <= 1.0).float().mean())


def _ckpt_worker(rank, world, port, path, out_q):
    _env(rank, world, port)
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed("cpu")
    eng = TrainEngine(_model(), info, lr=1e-2, weight_decay=0.1, bucket_mb=0.01, zero=1)
    for step in range(2):
        eng.train_step([_batch(rank, step)])
    eng.sync_params()
    eng.gather_optimizer_state()
    if rank == 0:
        torch.save({"model": eng.model.state_dict(), "optimizer": eng.state_dict()}, path)
    out_q.put((rank, eng.flat.numel))
    cleanup()


def test_zero1_checkpoint_resumes_on_one_rank_without_zero(tmp_path):
    """A checkpoint written by ZeRO-1 on 3 ranks (flat buffer padded to 3 x 64) loads into a single-process,
    unsharded engine (padded to 64) and into a 2-rank-sized layout: the optimizer buffers are saved trimmed to
    the parameters' extent (``flat.used``), so only the zero tail differs."""
    path = str(tmp_path / "z.pt")
    res = _spawn(_ckpt_worker, 3, path)
    ck = torch.load(path, weights_only=True)
    from bpe_transformer.train.engine import TrainEngine

    model = _model()
    eng = TrainEngine(model, lr=1e-2, weight_decay=0.1)
    assert eng.flat.numel != res[0], "the test needs layouts of different padded lengths"
    model.load_state_dict(ck["model"])
    eng.load_state_dict(ck["optimizer"])
    u = eng.flat.used
    assert ck["optimizer"]["master"].numel() == u
    torch.testing.assert_close(eng.opt.master[:u], ck["optimizer"]["master"])
    assert bool((eng.opt.exp_avg[u:] == 0).all())
    eng.train_step([_batch(0, 5)])  # and it trains on
    assert torch.isfinite(eng.flat.data).all()


def test_fp32_grad_accumulation_exact_where_bf16_rounds():
    """grad_accum = 4 on a bf16 model (CPU, autograd path): with the fp32 flat gradient buffer (each micro-batch's
    bf16 gradient folded into fp32 by the post-accumulate hook) the accumulated gradient equals the exact sum of
    the four micro-batch gradients; the bf16 buffer rounds the running sum at every micro-batch."""
    from bpe_transformer.optim.flat import FlatParameters

    micro = [_batch(r, 0) for r in range(4)]
    # exact reference: the same bf16 model's per-micro-batch gradients, summed in fp64
    model = _model(torch.bfloat16)
    ref = None
    for x, y in micro:
        model.zero_grad(set_to_none=True)
        (model.loss(x, y) / 4).backward()
        g = torch.cat([p.grad.reshape(-1).double() for p in model.parameters()])
        ref = g if ref is None else ref + g

    errs = {}
    for gdt in (torch.bfloat16, torch.float32):
        model = _model(torch.bfloat16)
        flat = FlatParameters.from_module(model, grad_dtype=gdt)
        for x, y in micro:
            (model.loss(x, y) / 4).backward()
        g = torch.cat([flat.grad[s.offset : s.offset + s.numel].double() for s in flat.slots])
        errs[gdt] = float((g - ref).norm() / ref.norm())
        if gdt == torch.float32:
            assert all(p.grad is None for p in model.parameters())  # folded into the flat buffer and released
    assert errs[torch.float32] < 1e-6, errs
    assert errs[torch.bfloat16] > 20 * errs[torch.float32], errs
