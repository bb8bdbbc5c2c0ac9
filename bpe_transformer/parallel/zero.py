"""Sharded data parallelism (ZeRO stage 1): reduce-scatter gradients, update a 1/N shard, all-gather weights.

Same flat-buffer design as :class:`~bpe_transformer.parallel.ddp.BucketedAllReduce`, with the optimizer work
divided over the ranks:

  * Buckets are fixed-size element ranges of the flat gradient buffer cut from the TOP (the LM head, whose
    gradient backward produces first) down, each a multiple of ``world x 64`` elements
    (``FlatParameters(pad_to=world * 64)`` pads the tail), so every bucket splits into ``world`` equal,
    64-aligned pieces.  Rank r owns piece r of every bucket.  A parameter may straddle two buckets; a bucket
    launches when every parameter overlapping it has its gradient.
  * Backward: per bucket, one in-place RCCL ``reduce_scatter_tensor`` (AVG) on RCCL's stream, overlapped with
    the rest of the backward.  It moves half the bytes of the all-reduce, so the bucket left exposed after
    the last gradient (the embedding's) costs half as much.
  * Step: the gradient norm is the sum of the ranks' piece norms (one 4-byte all-reduce, on the device); the
    AdamW kernels touch only the owned pieces -- 1/N of the optimizer's HBM traffic (26 bytes per parameter
    per step: fp32 master, two moments, bf16 grad and weight).
  * Then one in-place ``all_gather_into_tensor`` per bucket re-assembles the bf16 weights, issued in FORWARD
    order and waited lazily: the model calls :meth:`wait_params` for each module right before it reads that
    module's weights (``TransformerLM._bpe_param_fence``), so the gather of layer i+1 runs while layer i
    computes.  Anything else that reads the weights between steps calls :meth:`wait_all_params` first
    (``TrainEngine.sync_params``).

Optimizer state stays full-size on every rank (288 GB of HBM makes capacity a non-issue for the configs
here); only the owned pieces are current until :meth:`gather_optimizer_state` (collective, before a
checkpoint) makes all of it current, so checkpoints keep the unsharded format and load on any world size.

On gloo (CPU tests, and the 2-ranks-on-one-GPU test) a bucket is all-reduced instead of reduce-scattered, and
the weights are gathered as an all-reduce of a zero-filled bucket; the ownership, optimizer and fencing logic
is the same code.
"""

from __future__ import annotations

from contextlib import contextmanager

import torch
import torch.distributed as dist
from torch import Tensor, nn

from ..ops.optim import grad_norm
from ..optim.flat import ALIGN, FlatAdamW, FlatParameters


class ShardedDataParallel:
    sharded = True

    def __init__(self, flat: FlatParameters, bucket_mb: float = 64.0, process_group=None):
        assert dist.is_initialized(), "sharded data parallelism needs an initialised process group"
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self._nccl = dist.get_backend(process_group) == "nccl"
        self.enabled = True
        n = flat.numel
        unit = self.world * ALIGN
        if n % unit:
            raise ValueError(f"flat buffer of {n} elements does not split into {self.world} x {ALIGN}-element "
                             "pieces: build it with FlatParameters(..., pad_to=world * ALIGN)")
        bsz = max(unit, int(bucket_mb * (1 << 20)) // flat.grad.element_size() // unit * unit)
        self.buckets: list[tuple[int, int]] = []  # launch (= backward) order: highest offsets first
        top = n
        while top > 0:
            self.buckets.append((max(0, top - bsz), top))
            top = self.buckets[-1][0]
        self.pieces = [(s + self.rank * ((e - s) // self.world), s + (self.rank + 1) * ((e - s) // self.world))
                       for s, e in self.buckets]
        slots = flat.slots
        ends = [slots[i + 1].offset if i + 1 < len(slots) else n for i in range(len(slots))]
        self._param_buckets: dict[int, list[int]] = {}
        members = [0] * len(self.buckets)
        for sl, end in zip(slots, ends):
            bs = [b for b, (s, e) in enumerate(self.buckets) if s < end and sl.offset < e]
            self._param_buckets[id(sl.param)] = bs
            for b in bs:
                members[b] += 1
        self._members = members
        self._pending = list(members)
        self._seen: set[int] = set()
        self._rs: list = [None] * len(self.buckets)
        self._ag: list = [None] * len(self.buckets)
        self._ag_tmp: list = [None] * len(self.buckets)
        self._module_buckets: dict[int, list[int]] = {}
        self._hooks = []
        for sl in slots:
            self._hooks.append(sl.param.register_post_accumulate_grad_hook(self._on_grad))
            sl.param._bpe_grad_ready = self._on_grad

    # -- backward: reduce-scatter ------------------------------------------
    def _on_grad(self, p: torch.Tensor) -> None:
        # idempotent per backward (fused kernels notify, then AccumulateGrad fires too: parallel/ddp.py)
        if not self.enabled or id(p) in self._seen:
            return
        self._seen.add(id(p))
        for b in self._param_buckets[id(p)]:
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)

    def _launch(self, b: int) -> None:
        if self._rs[b] is not None:
            return
        s, e = self.buckets[b]
        ps, pe = self.pieces[b]
        full = self.flat.grad[s:e]

        def issue():
            if self._nccl:  # in place: the output is this rank's piece of the input
                return dist.reduce_scatter_tensor(self.flat.grad[ps:pe], full, op=dist.ReduceOp.AVG,
                                                  group=self.pg, async_op=True)
            return dist.all_reduce(full, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

        self._rs[b] = issue()

    def start(self) -> None:
        """Call before each backward that should reduce."""
        self._pending = list(self._members)
        self._seen = set()
        self._rs = [None] * len(self.buckets)

    def finish(self) -> None:
        """Launch buckets whose hooks never fired, then order the compute stream after every reduce-scatter.
        Afterwards only this rank's pieces of ``flat.grad`` hold the averaged gradient."""
        for b in range(len(self.buckets)):
            if self._rs[b] is None:
                self._launch(b)
        for w in self._rs:
            w.wait()
        if not self._nccl:
            for ps, pe in self.pieces:
                self.flat.grad[ps:pe].div_(self.world)
        self._rs = [None] * len(self.buckets)

    @contextmanager
    def no_sync(self):
        """Gradient accumulation: skip the collectives for the micro-batches inside."""
        prev = self.enabled
        self.enabled = False
        try:
            yield
        finally:
            self.enabled = prev

    # -- step --------------------------------------------------------------
    def shard_ranges(self) -> list[tuple[int, int]]:
        return list(self.pieces)

    @torch.no_grad()
    def clip_coef(self, max_norm: float) -> tuple[Tensor, Tensor]:
        """Global gradient L2 norm from the owned pieces (one scalar all-reduce) and the clip coefficient
        (-1 = non-finite norm: the AdamW kernels skip the step), both on the device."""
        g = self.flat.grad
        local, _ = grad_norm([g[ps:pe] for ps, pe in self.pieces])
        sq = (local.float() * local.float()).reshape(1)
        dist.all_reduce(sq, op=dist.ReduceOp.SUM, group=self.pg)
        norm = sq.sqrt()[0]
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        coef = torch.where(torch.isfinite(norm), coef, torch.full_like(coef, -1.0))
        return norm, coef

    # -- weights: all-gather, waited lazily --------------------------------
    @torch.no_grad()
    def gather_params(self) -> None:
        """Launch the weight all-gathers (forward order) after the optimizer updated the owned pieces."""
        data = self.flat.data
        for b in reversed(range(len(self.buckets))):
            s, e = self.buckets[b]
            ps, pe = self.pieces[b]
            if self._nccl:
                self._ag[b] = dist.all_gather_into_tensor(data[s:e], data[ps:pe], group=self.pg, async_op=True)
            else:  # gloo: all-reduce of a bucket that is zero outside this rank's piece (exact in any dtype)
                tmp = torch.zeros_like(data[s:e])
                tmp[ps - s : pe - s].copy_(data[ps:pe])
                self._ag_tmp[b] = tmp
                self._ag[b] = dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def _wait_bucket(self, b: int) -> None:
        w = self._ag[b]
        if w is None:
            return
        w.wait()
        self._ag[b] = None
        tmp = self._ag_tmp[b]
        if tmp is not None:
            s, e = self.buckets[b]
            self.flat.data[s:e].copy_(tmp)
            self._ag_tmp[b] = None

    def wait_params(self, module: nn.Module) -> None:
        """Make the current stream wait for the all-gathers covering ``module``'s weights (no host sync on
        RCCL).  Cheap when nothing is pending; the bucket list per module is cached."""
        bs = self._module_buckets.get(id(module))
        if bs is None:
            acc: set[int] = set()
            for p in module.parameters():
                acc.update(self._param_buckets.get(id(p), ()))
            bs = self._module_buckets[id(module)] = sorted(acc, reverse=True)  # forward order
        for b in bs:
            self._wait_bucket(b)

    def wait_all_params(self) -> None:
        for b in reversed(range(len(self.buckets))):
            self._wait_bucket(b)

    # -- checkpoints / checks ----------------------------------------------
    @torch.no_grad()
    def gather_optimizer_state(self, opt: FlatAdamW) -> None:
        """Collective: make the full fp32 master / moment buffers current on every rank."""
        self.wait_all_params()
        bufs = [opt.exp_avg, opt.exp_avg_sq] + ([opt.master] if opt.master is not self.flat.data else [])
        for buf in bufs:
            for (s, e), (ps, pe) in zip(self.buckets, self.pieces):
                if self._nccl:
                    dist.all_gather_into_tensor(buf[s:e], buf[ps:pe].clone(), group=self.pg)
                else:
                    tmp = torch.zeros_like(buf[s:e])
                    tmp[ps - s : pe - s].copy_(buf[ps:pe])
                    dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=self.pg)
                    buf[s:e].copy_(tmp)

    @torch.no_grad()
    def check_consistency(self, what: str = "data") -> None:
        """Raise if the ranks' weights differ (after the all-gathers).  ``what="grad"`` is a no-op: after the
        reduce-scatter each rank holds a different piece of the gradient by design."""
        if what != "data":
            return
        self.wait_all_params()
        d = self.flat.data
        sums = torch.stack([d[s:e].sum(dtype=torch.float64) for s, e in self.buckets]
                           + [d[s:e].abs().sum(dtype=torch.float64) for s, e in self.buckets])
        both = torch.cat([sums, -sums])
        dist.all_reduce(both, op=dist.ReduceOp.MAX, group=self.pg)
        n = sums.numel()
        bad = (both[:n] != -both[n:]).nonzero().flatten().tolist()
        if bad:
            raise RuntimeError(f"sharded data-parallel weight divergence across ranks in bucket(s) "
                               f"{sorted({i % len(self.buckets) for i in bad})}")

    @torch.no_grad()
    def broadcast_parameters(self, src: int = 0) -> None:
        dist.broadcast(self.flat.data, src=src, group=self.pg)

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
