"""Data parallelism: bucketed gradient all-reduce overlapped with backward.

MI355X / RCCL-over-xGMI design:
  * Gradients live in ONE flat buffer (:class:`~bpe_transformer.optim.flat.FlatParameters`);
    a bucket is a contiguous slice of it, so a collective needs no
    flatten/unflatten copies.
  * Buckets are formed walking parameters in REVERSE registration order (the
    order backward produces them: LM head first, embedding last) and closed
    at ``bucket_mb``.  Each parameter has a post-accumulate-grad hook; when
    the last gradient of a bucket lands, the bucket's all-reduce is launched
    asynchronously.  RCCL runs it on its own internal HIP stream (ordered
    after the producing kernels by an event), so it overlaps the rest of the
    backward; ``finish()`` only makes the compute stream wait on the
    collectives before the optimizer (no host sync).
  * Bucket size is chosen for xGMI: each GPU has 7 point-to-point links; ring
    collectives are per-link bound, so fewer, larger buckets (tens of MB)
    amortise launch latency while still leaving several buckets to overlap.
  * Averaging uses ``ReduceOp.AVG`` on RCCL (no extra scaling pass); on gloo
    (CPU tests) SUM + divide.
  * ``comm_dtype``: the wire / reduction dtype when it differs from the gradient buffer's.  bf16 gradients
    reduced as fp32 (each bucket cast into an fp32 staging slice before its collective and back after the wait)
    are summed across the ring without a bf16 rounding at every hop, for 2x the bytes; fp32 gradients (grad
    accumulation) reduced as bf16 halve the bytes.  Default: the gradient dtype.
"""

from __future__ import annotations

from contextlib import contextmanager

import torch
import torch.distributed as dist

from ..optim.flat import FlatParameters


class BucketedAllReduce:
    def __init__(self, flat: FlatParameters, bucket_mb: float = 64.0, process_group=None, overlap: bool = True,
                 average: bool = True, comm_dtype: torch.dtype | None = None):
        self.flat = flat
        self.comm_dtype = comm_dtype or flat.grad.dtype
        # staging buffer for a wire dtype other than the gradient's (one flat buffer, sliced like the buckets)
        self._cbuf = (torch.empty(flat.numel, dtype=self.comm_dtype, device=flat.grad.device)
                      if self.comm_dtype != flat.grad.dtype else None)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.average = average
        self.overlap = overlap
        self.enabled = True
        self._use_avg = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
        elem = flat.grad.element_size()
        limit = int(bucket_mb * (1 << 20))
        slots = flat.slots
        ends = [slots[i + 1].offset if i + 1 < len(slots) else flat.numel for i in range(len(slots))]
        self.buckets: list[tuple[int, int]] = []  # [start, end) in elements, in launch order
        self.bucket_of: dict[int, int] = {}
        members: list[list[int]] = []
        cur: list[int] = []
        cur_bytes = 0
        for i in reversed(range(len(slots))):
            cur.append(i)
            cur_bytes += (ends[i] - slots[i].offset) * elem
            if cur_bytes >= limit:
                members.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            members.append(cur)
        for b, mem in enumerate(members):
            self.buckets.append((slots[min(mem)].offset, ends[max(mem)]))
            for i in mem:
                self.bucket_of[id(slots[i].param)] = b
        self._members = [len(m) for m in members]
        self._pending = list(self._members)
        self._seen: set[int] = set()
        self._works: list = [None] * len(self.buckets)
        self._hooks = []
        if overlap and self.world > 1:
            for s in slots:
                self._hooks.append(s.param.register_post_accumulate_grad_hook(self._on_grad))
                # kernels that accumulate into param.main_grad themselves call this instead
                s.param._bpe_grad_ready = self._on_grad

    # -- hooks -------------------------------------------------------------
    def _on_grad(self, p: torch.Tensor) -> None:
        # Idempotent per backward: a parameter whose gradient a fused kernel writes into main_grad notifies
        # right after that write, and its AccumulateGrad node still runs afterwards (with an undefined grad)
        # and fires the post-accumulate hook a second time -- counting both would launch the bucket's
        # collective before its other members' gradients exist.
        if not self.enabled or id(p) in self._seen:
            return
        self._seen.add(id(p))
        b = self.bucket_of[id(p)]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def _launch(self, b: int) -> None:
        if self._works[b] is not None:
            return
        s, e = self.buckets[b]
        view = self.flat.grad[s:e]
        if self._cbuf is not None:
            # every gradient is produced on the current (compute) stream, so this copy -- and the collective,
            # which RCCL orders after the current stream -- follow all writes to the bucket
            self._cbuf[s:e].copy_(view)
            view = self._cbuf[s:e]
        op = dist.ReduceOp.AVG if (self.average and self._use_avg) else dist.ReduceOp.SUM
        self._works[b] = dist.all_reduce(view, op=op, group=self.pg, async_op=True)

    # -- step API ----------------------------------------------------------
    def start(self) -> None:
        """Call before each backward that should all-reduce."""
        self._pending = list(self._members)
        self._seen = set()
        self._works = [None] * len(self.buckets)

    def finish(self) -> None:
        """Launch buckets whose hooks never fired, then order the compute stream after every collective."""
        if self.world <= 1:
            return
        for b in range(len(self.buckets)):
            if self._works[b] is None:
                self._launch(b)
        for w in self._works:
            w.wait()
        if self._cbuf is not None:
            self.flat.grad.copy_(self._cbuf)
        if self.average and not self._use_avg:
            self.flat.grad.div_(self.world)
        self._works = [None] * len(self.buckets)

    @contextmanager
    def no_sync(self):
        """Gradient accumulation: skip the collectives for the micro-batches inside."""
        prev = self.enabled
        self.enabled = False
        try:
            yield
        finally:
            self.enabled = prev

    # -- race / divergence detection ---------------------------
    @torch.no_grad()
    def check_consistency(self, what: str = "grad") -> None:
        """Raise if the ranks do not hold bit-identical gradients (``what="grad"``, call after :meth:`finish`)
        or weights (``"data"``, after the optimizer step).

        Data parallelism keeps replicas identical only if every bucket's collective saw every member's final
        gradient; a collective launched too early (an ordering race) or a rank that skipped one shows up as a
        checksum mismatch.  Costs one small all-reduce of per-bucket fp64 checksums (MAX of [c, -c] gives the
        max and -min in one collective); it synchronises the host to raise, so enable it every N steps
        (``TrainConfig.ddp_check_every``), not every step.
        """
        if self.world <= 1:
            return
        buf = self.flat.grad if what == "grad" else self.flat.data
        sums = torch.stack([buf[s:e].sum(dtype=torch.float64) for s, e in self.buckets]
                           + [buf[s:e].abs().sum(dtype=torch.float64) for s, e in self.buckets])
        both = torch.cat([sums, -sums])
        dist.all_reduce(both, op=dist.ReduceOp.MAX, group=self.pg)
        n = sums.numel()
        hi, lo = both[:n], -both[n:]
        bad = (hi != lo).nonzero().flatten().tolist()
        if bad:
            nb = len(self.buckets)
            idx = sorted({i % nb for i in bad})
            raise RuntimeError(f"data-parallel {what} divergence across ranks in bucket(s) {idx} "
                               f"(checksum spread {float((hi - lo).abs().max()):.3e})")

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks.clear()

    @torch.no_grad()
    def broadcast_parameters(self, src: int = 0) -> None:
        """Make every rank start from rank ``src``'s weights (one collective over the flat buffer)."""
        if self.world > 1:
            dist.broadcast(self.flat.data, src=src, group=self.pg)
