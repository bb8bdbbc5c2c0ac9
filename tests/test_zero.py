"""Sharded data parallelism (``parallel/zero.py``, ZeRO-1) on the CPU (gloo).

Ranks reduce their gradient buckets, each updates only its piece of every bucket, and the weights are
re-assembled by all-gathers that the next forward waits for module by module.  The result must equal the
unsharded data-parallel engine on the same ranks and batches -- weights, fp32 master and both AdamW moments
(after ``gather_optimizer_state``) -- with weight decay on (segment x shard intersections), clipping active,
uneven bucket splits (world 3) and gradient accumulation.
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


def _batch(rank: int, step: int, micro: int):
    g = torch.Generator().manual_seed(100 + 17 * rank + 1000 * step + 7 * micro)
    x = torch.randint(0, 200, (2, 32), generator=g)
    return x, torch.roll(x, -1, 1)


def _worker(rank, world, port, zero, accum, bucket_mb, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from bpe_transformer.parallel import cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed("cpu")
    eng = TrainEngine(_model(), info, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5, bucket_mb=bucket_mb, zero=zero,
                      ddp_check_every=2)
    norms = []
    for step in range(3):
        eng.train_step([_batch(rank, step, m) for m in range(accum)])
        norms.append(float(eng.last_grad_norm))
    eng.sync_params()
    if zero:
        try:
            eng.state_dict()
            raise AssertionError("state_dict() must refuse stale sharded optimizer state")
        except RuntimeError:
            pass
    eng.gather_optimizer_state()
    sd = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in eng.state_dict().items()}
    nb = len(eng.ddp.buckets)
    pieces = list(getattr(eng.ddp, "pieces", []))
    out = (rank, eng.flat.data.numpy().copy(), sd["master"].numpy().copy(), sd["exp_avg"].numpy().copy(),
           sd["exp_avg_sq"].numpy().copy(), int(sd["step"]), norms, nb, pieces, eng.flat.numel)
    # resume: a fresh engine loading the gathered (unsharded-format) state continues exactly like this one
    model2 = _model()
    eng2 = TrainEngine(model2, info, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5, bucket_mb=bucket_mb, zero=zero)
    model2.load_state_dict(eng.model.state_dict())
    eng2.load_state_dict(sd)
    eng.train_step([_batch(rank, 9, 0)])
    eng2.train_step([_batch(rank, 9, 0)])
    eng.sync_params()
    eng2.sync_params()
    resumed_equal = bool(torch.equal(eng.flat.data, eng2.flat.data))
    out_q.put(out + (resumed_equal,))
    cleanup()


def _run(world, zero, accum=1, bucket_mb=0.01):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, zero, accum, bucket_mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=240) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,accum", [(2, 1), (3, 2)])
def test_zero1_matches_unsharded_dp(world, accum):
    z = _run(world, 1, accum)
    d = _run(world, 0, accum)
    assert z[0][6] > 2, "expected several buckets"
    for r in range(1, world):
        for k in range(4):  # weights, master, moments: identical on every rank after the gathers
            assert (z[r][k] == z[0][k]).all(), f"rank {r} differs in field {k}"
    assert z[0][4] == d[0][4] == 3
    # the layouts differ only in the zero tail (pad_to); the moments match tightly, the weights to the
    # reduction-order noise of 3-rank gloo rings with different bucket cuts, which Adam amplifies where v ~ 0
    # (measured: moments <= 1e-8, weights <= 5e-5 at 3 of 35k elements)
    for k, name, atol in [(0, "data", 2e-4), (1, "master", 2e-4), (2, "exp_avg", 1e-7), (3, "exp_avg_sq", 1e-9)]:
        a, b = torch.from_numpy(z[0][k]), torch.from_numpy(d[0][k])
        m = min(a.shape[0], b.shape[0])
        torch.testing.assert_close(a[:m], b[:m], atol=atol, rtol=1e-5, msg=name)
        assert float((a[:m] - b[:m]).abs().gt(1e-6).float().mean()) < 1e-3, name
    for gz, gd in zip(z[0][5], d[0][5]):
        assert abs(gz - gd) <= 1e-5 * max(1.0, gd), (gz, gd)
    # ownership: the ranks' pieces are 64-aligned, equal per bucket, disjoint, and tile the padded buffer
    numel = z[0][8]
    assert numel % (64 * world) == 0
    cover = torch.zeros(numel, dtype=torch.int32)
    for r in range(world):
        for s, e in z[r][7]:
            assert s % 64 == 0 and e % 64 == 0
            cover[s:e] += 1
    assert bool((cover == 1).all())
    # resume from the gathered state reproduces the next step bit for bit, on both engines
    assert all(z[r][9] for r in range(world)) and all(d[r][9] for r in range(world))


def _trainer_worker(rank, world, port, zero, ckdir, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from bpe_transformer.models import get_preset
    from bpe_transformer.parallel import cleanup
    from bpe_transformer.train.config import TrainConfig
    from bpe_transformer.train.trainer import Trainer

    cfg = TrainConfig(model=get_preset("ts-tests", vocab_size=256, context_length=16), batch_size=4, max_iters=4,
                      device="cpu", log_every=2, ckpt_every=4, ckpt_dir=ckdir, zero=zero)
    cfg.optim.warmup_iters = 1
    cfg.data.synthetic_tokens = 20_000
    out = Trainer(cfg).fit()
    out_q.put((rank, out["final_loss"]))
    cleanup()


def test_zero1_trainer_checkpoint_is_unsharded(tmp_path):
    """Trainer with zero=1 on 2 ranks: every rank joins the gathers, rank 0 writes the full optimizer state,
    and the checkpoint matches the unsharded data-parallel run's."""
    cks = {}
    for zero in (0, 1):
        port = _free_port()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ck = str(tmp_path / f"z{zero}")
        procs = [ctx.Process(target=_trainer_worker, args=(r, 2, port, zero, ck, q)) for r in range(2)]
        for p in procs:
            p.start()
        losses = [q.get(timeout=240) for _ in range(2)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert all(loss == loss for _, loss in losses)
        cks[zero] = torch.load(os.path.join(ck, "ckpt_00000004.pt"), weights_only=True)
    a, b = cks[1]["optimizer"], cks[0]["optimizer"]
    assert a["step"] == b["step"] == 4
    for k in ("master", "exp_avg", "exp_avg_sq"):
        m = min(a[k].numel(), b[k].numel())
        torch.testing.assert_close(a[k][:m], b[k][:m], atol=2e-4, rtol=1e-4, msg=k)
    for k, v in cks[0]["model"].items():
        torch.testing.assert_close(cks[1]["model"][k], v, atol=2e-4, rtol=1e-4, msg=k)
