"""The training step engine shared by the trainer loop and ``bench.py``.

One step = (micro-batches of) fused forward + LM-head/CE -> backward with the
bucketed RCCL all-reduce overlapping it -> global-norm clip (coefficient kept
on the device) -> one flat fused-AdamW pass writing fp32 master + bf16 weights.
Nothing in the step synchronises the host; the returned loss is a device
tensor.

Reference: the reference implies this step only through its test utilities
(``tests/test_optimizer.py:18-25``, ``tests/adapters.py:401-542``).
"""

from __future__ import annotations

from contextlib import nullcontext

import torch
from torch import Tensor, nn

from ..optim.flat import FlatAdamW, FlatParameters
from ..optim.flat import ALIGN
from ..parallel.ddp import BucketedAllReduce
from ..parallel.dist import DistInfo
from ..parallel.zero import ShardedDataParallel


class TrainEngine:
    def __init__(
        self,
        model: nn.Module,
        dist_info: DistInfo | None = None,
        lr: float = 3e-4,
        betas=(0.9, 0.95),
        eps: float = 1e-8,
        weight_decay: float = 0.1,
        max_grad_norm: float | None = 1.0,
        bucket_mb: float = 64.0,
        time_phases: bool = False,
        ddp_check_every: int = 0,
        zero: int = 0,
        grad_dtype: torch.dtype | None = None,
        comm_dtype: torch.dtype | None = None,
    ):
        """``grad_dtype``: dtype of the flat gradient buffer (default: the parameters', bf16 on the GPU path);
        fp32 keeps the weight gradients -- and their sum over grad-accumulation micro-batches -- unrounded
        (the dW kernels write fp32 through their partial slab).  ``comm_dtype``: the data-parallel all-reduce
        dtype (default: the gradient dtype; ``parallel/ddp.py``)."""
        self.model = model
        self.dist = dist_info or DistInfo()
        # zero=1: sharded data parallelism (parallel/zero.py) -- reduce-scatter, 1/N of the AdamW work,
        # all-gather of the weights overlapped with the next forward
        # (a one-rank job gets the sharded path only inside an explicitly initialised process group: tests of
        # the RCCL calls on one GPU)
        self.zero = int(zero) if (self.dist.world_size > 1 or (zero and torch.distributed.is_initialized())) else 0
        pad = self.dist.world_size * ALIGN if self.zero else ALIGN
        self.flat = FlatParameters.from_module(model, grad_dtype=grad_dtype, pad_to=pad)
        for slot in self.flat.slots:  # fused blocks accumulate weight grads straight into the flat buffer
            slot.param.main_grad = self.flat.grad_view(slot).view_as(slot.param)
        self.opt = FlatAdamW(self.flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.max_grad_norm = max_grad_norm
        self.ddp = None
        if self.dist.world_size > 1 or self.zero:
            self.ddp = (ShardedDataParallel(self.flat, bucket_mb=bucket_mb) if self.zero
                        else BucketedAllReduce(self.flat, bucket_mb=bucket_mb, comm_dtype=comm_dtype))
        if self.ddp is not None:
            self.ddp.broadcast_parameters(0)
            self.opt.master.copy_(self.flat.data)  # keep fp32 master == broadcast weights
        self._fenced = False
        self._opt_state_current = True  # sharded DP: False from a step until gather_optimizer_state()
        if self.zero:
            self.opt.set_shard(self.ddp.shard_ranges())
            # the model waits for each module's weight all-gather right before reading it; a model without
            # that hook waits for all of them at the start of the next step instead
            if hasattr(model, "_bpe_param_fence"):
                model._bpe_param_fence = self.ddp.wait_params
                self._fenced = True
        self.last_grad_norm: Tensor | None = None
        # DP race / divergence detector: every N steps compare per-bucket gradient and weight checksums across
        # ranks (parallel/ddp.py check_consistency; raises on mismatch)
        self.ddp_check_every = ddp_check_every
        self.steps_done = 0
        # phase timing (SURVEY §5 tracing): device events around forward / backward / exposed all-reduce wait /
        # clip + optimizer, recorded every step and only read (one host sync) when phase_times() is called
        self.time_phases = time_phases and torch.cuda.is_available() and self.flat.data.is_cuda
        self._ev: dict[str, list] = {}

    def _mark(self, name: str) -> None:
        if self.time_phases:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._ev.setdefault(name, []).append(e)

    def phase_times(self) -> dict[str, float]:
        """Mean milliseconds per step of each phase since the last call (synchronises the device)."""
        if not self.time_phases or "start" not in self._ev:
            return {}
        torch.cuda.synchronize()
        order = ["start", "fwd", "bwd", "comm", "opt"]
        out: dict[str, float] = {}
        n = len(self._ev["start"])
        for a, b in zip(order, order[1:]):
            if a in self._ev and b in self._ev and len(self._ev[b]) == n:
                out[f"{b}_ms"] = sum(x.elapsed_time(y) for x, y in zip(self._ev[a], self._ev[b])) / n
        self._ev.clear()
        return out

    def train_step(self, batches: list[tuple[Tensor, Tensor]], lr: float | None = None) -> Tensor:
        """Run one optimizer step over ``batches`` (gradient accumulation when > 1).

        Returns the mean loss as a 0-dim device tensor (no host sync).
        """
        self.model.train()
        self._mark("start")
        if self.zero and not self._fenced:
            self.ddp.wait_all_params()
        self.flat.grad.zero_()
        n = len(batches)
        total = None
        for i, (x, y) in enumerate(batches):
            last = i == n - 1
            if self.ddp is not None and last:
                self.ddp.start()
            ctx = self.ddp.no_sync() if (self.ddp is not None and not last) else nullcontext()
            with ctx:
                loss = self.model.loss(x, y)
                if last:
                    self._mark("fwd")
                (loss / n if n > 1 else loss).backward()
            total = loss.detach() if total is None else total + loss.detach()
        self._mark("bwd")
        if self.ddp is not None:
            self.ddp.finish()
        check = self.ddp is not None and self.ddp_check_every > 0 and self.steps_done % self.ddp_check_every == 0
        if check:
            self.ddp.check_consistency("grad")
        self._mark("comm")
        coef = None
        if self.max_grad_norm is not None and self.max_grad_norm > 0:
            if self.zero:
                norm, coef = self.ddp.clip_coef(self.max_grad_norm)
            else:
                norm, coef = self.opt.clip_grad_norm(self.max_grad_norm)
            self.last_grad_norm = norm
        self.opt.step(lr, coef)
        if self.zero:
            self.ddp.gather_params()  # waited per module by the next forward (or sync_params)
            self._opt_state_current = False
        if check:
            self.ddp.check_consistency("data")
        self.steps_done += 1
        self._mark("opt")
        states = self.model.fp8_states() if hasattr(self.model, "fp8_states") else []
        for fp8 in states:
            if self.ddp is not None:
                # identical scales on every rank: amax bit patterns order like the (non-negative) floats
                torch.distributed.all_reduce(fp8.amax, op=torch.distributed.ReduceOp.MAX)
            fp8.update()
        return total / n if n > 1 else total

    def sync_params(self) -> None:
        """Wait for in-flight weight all-gathers (sharded DP); call before reading the weights outside a
        forward (evaluation through other code paths, checkpoints, comparisons).  No-op otherwise."""
        if self.zero:
            self.ddp.wait_all_params()

    def gather_optimizer_state(self) -> None:
        """Collective on every rank (sharded DP): make the full optimizer state current before a checkpoint.
        No-op otherwise."""
        if self.zero:
            self.ddp.gather_optimizer_state(self.opt)
            self._opt_state_current = True

    def state_dict(self) -> dict:
        if not self._opt_state_current:
            raise RuntimeError("sharded data parallelism: only this rank's pieces of the optimizer state are "
                               "current; call gather_optimizer_state() on every rank before state_dict()")
        return self.opt.state_dict()

    def load_state_dict(self, sd: dict) -> None:
        self.opt.load_state_dict(sd)
