"""Data-parallel correctness on the CPU (gloo, 2 processes).

The bucketed all-reduce (``parallel.ddp.BucketedAllReduce``) fires from
post-accumulate-grad hooks during backward.  Two ranks training on different
micro-batches must end bit-for-bit identical to each other and equal (to
float tolerance) a single process that trains on the concatenated batch.
"""

from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.dist


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    from bpe_transformer.models import TransformerLM

    torch.manual_seed(0)
    return TransformerLM(200, 32, 32, 2, 2, 64)


def _batches(rank: int):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randint(0, 200, (2, 32), generator=g)
    return x, torch.roll(x, -1, 1)


def _worker(rank, world, port, bucket_mb, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed("cpu")
    model = _model()
    eng = TrainEngine(model, info, lr=1e-2, weight_decay=0.0, max_grad_norm=1.0, bucket_mb=bucket_mb)
    assert len(eng.ddp.buckets) >= (2 if bucket_mb < 0.05 else 1)
    for _ in range(3):
        eng.train_step([_batches(rank)])
    # numpy copies travel by value; torch tensors would go through fd sharing whose
    # listener dies with this process (flaky under pytest-xdist)
    out_q.put((rank, eng.flat.data.numpy().copy(), eng.flat.grad.numpy().copy()))
    cleanup()


@pytest.mark.parametrize("bucket_mb", [0.01, 64.0])
def test_dp2_matches_single_process(bucket_mb):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(d), torch.from_numpy(g))) for r, d, g in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.equal(res[0][0], res[1][0]), "ranks diverged"
    # single-process reference: the mean loss over both ranks' micro-batches == one batch of 4
    from bpe_transformer.train.engine import TrainEngine

    model = _model()
    eng = TrainEngine(model, lr=1e-2, weight_decay=0.0, max_grad_norm=1.0)
    x0, y0 = _batches(0)
    x1, y1 = _batches(1)
    for _ in range(3):
        eng.train_step([(torch.cat([x0, x1]), torch.cat([y0, y1]))])
    torch.testing.assert_close(res[0][0], eng.flat.data, atol=2e-5, rtol=1e-4)


def _launched(out_dir):
    import torch.distributed as dist

    from bpe_transformer.parallel import cleanup, init_distributed

    info = init_distributed("cpu")
    t = torch.tensor([float(info.rank + 1)])
    dist.all_reduce(t)
    with open(os.path.join(out_dir, f"rank{info.rank}.txt"), "w") as f:
        f.write(f"{info.world_size} {t.item()} {os.environ['MASTER_ADDR']}")
    cleanup()


def test_launcher_spawns_ranks(tmp_path):
    """parallel.launch: torchrun-style env in every rank, gloo collective across them."""
    from bpe_transformer.parallel.launch import launch

    launch(_launched, 2, str(tmp_path))
    for r in range(2):
        assert (tmp_path / f"rank{r}.txt").read_text() == "2 3.0 127.0.0.1"


def test_bucket_notifications_idempotent():
    """A parameter notified twice in one backward (fused main_grad write + its AccumulateGrad hook) must
    count once: the bucket's collective may only start when every member's gradient exists."""
    from bpe_transformer.optim.flat import FlatParameters
    from bpe_transformer.parallel.ddp import BucketedAllReduce

    flat = FlatParameters.from_module(_model())
    ar = BucketedAllReduce.__new__(BucketedAllReduce)
    BucketedAllReduce.__init__(ar, flat, bucket_mb=1e9, overlap=False)  # world 1: no hooks, one bucket
    launched = []
    ar._launch = lambda b: launched.append(b)
    ar.start()
    params = [s.param for s in flat.slots]
    for p in params[:-1]:
        ar._on_grad(p)
        ar._on_grad(p)  # the duplicate must not count
    assert launched == []
    ar._on_grad(params[-1])
    assert launched == [0]
    ar.start()
    assert ar._seen == set() and ar._pending == ar._members


def _check_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed("cpu")
    eng = TrainEngine(_model(), info, lr=1e-2, bucket_mb=0.01, ddp_check_every=1)
    eng.train_step([_batches(rank)])  # consistent: must not raise
    ok = True
    # inject a divergence: rank 1 perturbs its weights; the next check must catch it on every rank
    if rank == 1:
        with torch.no_grad():
            eng.flat.data[5] += 1.0
    try:
        eng.train_step([_batches(rank)])
        ok = False
    except RuntimeError as e:
        ok = "divergence" in str(e)
    out_q.put((rank, ok))
    cleanup()


def test_ddp_consistency_check_detects_divergence():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}



@pytest.mark.parametrize("zero", [0, 1])
def test_bench_contract_two_ranks_cpu(tmp_path, zero):
    """bench.py under torch.distributed.run with 2 ranks (gloo, CPU plumbing config) prints exactly one JSON line,
    from rank 0, with the whole-job numbers the driver's scaling run reads (n_gpus, dp2, global batch)."""
    import json
    import os
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "2", "--device", "cpu", "--model", "tinystories-17m", "--seq", "32", "--batch", "2",
           "--steps", "2", "--warmup", "1", "--zero", str(zero)]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1 and out["scaling"] == "weak"
    assert out["config"]["parallelism"] == ("dp2-zero1" if zero else "dp2") and out["config"]["global_batch"] == 4
    assert out["value"] > 0 and abs(out["value"] - 2 * 2 * 2 * 32 / (out["ms_per_step"] * 2 / 1000)) < 0.02 * out["value"]
    # the self-validation the first multi-GPU record carries: world size, backend, bucket layout, wire dtype and the
    # untimed replica-consistency step's verdict
    d = out["dist"]
    assert d["world_size"] == 2 and d["backend"] == "gloo" and d["buckets"] == len(d["bucket_mb"]) >= 1
    assert d["comm_dtype"] in ("float32", "bfloat16")
    assert d["consistency_check"] == ("data bit-identical across ranks" if zero else
                                      "grad+data bit-identical across ranks")


@pytest.mark.parametrize("zero", [0])
def test_bench_refuses_a_corrupted_replica(tmp_path, zero):
    """A replica whose weights were perturbed before the consistency step makes bench.py fail with the divergence
    error instead of printing a throughput record.  (Plain data parallelism only: under ZeRO-1 every rank's weights
    are re-gathered from the owners' shards each step, so a perturbed replica heals and the data check guards the
    all-gather itself.)"""
    import os
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "2", "--device", "cpu", "--model", "tinystories-17m", "--seq", "32", "--batch", "2",
           "--steps", "1", "--warmup", "1", "--zero", str(zero), "--debug-corrupt-rank", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode != 0
    assert "divergence" in r.stderr + r.stdout
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
