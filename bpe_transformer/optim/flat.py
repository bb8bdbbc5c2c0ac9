"""Flat parameter / gradient storage and the one-launch optimizer step.

MI355X-first design: all trainable parameters of the model live in ONE
contiguous buffer (each ``Parameter`` becomes a view into it) and all gradients
in ONE contiguous buffer laid out identically.  That buys:

  * the optimizer step is a handful of grid-stride launches over HBM
    (``FlatAdamW``), independent of the number of tensors;
  * gradient clipping is one two-stage reduction over one buffer, and its
    coefficient feeds the AdamW kernel on the device (no host sync);
  * data-parallel gradient buckets are plain slices of the flat gradient
    buffer, so bucketed RCCL all-reduces need no flatten/unflatten copies
    (``parallel.ddp``).

Parameters are packed in registration order, each starting at a 64-element
aligned offset (16-byte vector alignment for every kernel; padding stays 0).

A 2-D parameter may ask for zero ROW padding (``param._bpe_pad_rows = R``, or
``module.pad_rows = R`` on its module for :meth:`FlatParameters.from_module`):
its slot then reserves ``R x cols`` elements and the parameter is the first
``rows`` of them.  ``param._bpe_padded`` / ``param._bpe_padded_grad`` are the
``[R, cols]`` views.  The LM head uses this so the vocab dimension of its
GEMMs is a multiple of 256 (vocab 50257 is odd: an odd logits row stride
rules out the libraries' vector accesses).  The pad rows receive zero
gradients, so AdamW keeps them exactly zero.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import Tensor, nn

from ..ops.optim import count_adam_step, fused_adamw_step, grad_norm

ALIGN = 64


@dataclass
class Slot:
    name: str
    param: nn.Parameter
    offset: int
    numel: int


class FlatParameters:
    def __init__(self, named_params: list[tuple[str, nn.Parameter]], grad_dtype: torch.dtype | None = None,
                 pad_to: int = ALIGN):
        """``pad_to``: the total length is rounded up to a multiple of it (zero tail; sharded data parallelism
        needs buckets that split evenly over the ranks, ``parallel/zero.py``)."""
        assert named_params, "no parameters"
        dtypes = {p.dtype for _, p in named_params}
        devices = {p.device for _, p in named_params}
        assert len(dtypes) == 1 and len(devices) == 1, "flat buffers need one dtype and one device"
        self.dtype = dtypes.pop()
        self.device = devices.pop()
        self.slots: list[Slot] = []
        off = 0
        reserve: list[int] = []
        for name, p in named_params:
            n = p.numel()
            pad_rows = getattr(p, "_bpe_pad_rows", None)
            r = pad_rows * p.shape[1] if (pad_rows and p.dim() == 2 and pad_rows >= p.shape[0]) else n
            self.slots.append(Slot(name, p, off, n))
            reserve.append(r)
            off += (r + ALIGN - 1) // ALIGN * ALIGN
        self.used = off  # end of the last slot: the layout up to here does not depend on pad_to
        off = (off + pad_to - 1) // pad_to * pad_to
        self.numel = off
        self.data = torch.zeros(off, dtype=self.dtype, device=self.device)
        self.grad = torch.zeros(off, dtype=grad_dtype or self.dtype, device=self.device)
        # fp32 gradients for bf16 parameters: ``param.grad`` must match the parameter's dtype, so the flat fp32
        # slots are not attached as ``.grad``.  Kernels that know the flat buffer accumulate into
        # ``param.main_grad`` (set by the training engine) directly; a gradient that arrives through autograd's
        # AccumulateGrad is added into the fp32 slot by a post-accumulate hook and released (registered here,
        # before any data-parallel hook, so those see the slot already updated).
        self.split_grad = self.grad.dtype != self.dtype
        self._hooks = []
        with torch.no_grad():
            for s, r in zip(self.slots, reserve):
                view = self.data[s.offset : s.offset + s.numel].view_as(s.param)
                view.copy_(s.param.data)
                s.param.data = view
                if self.split_grad:
                    s.param.grad = None
                    self._hooks.append(s.param.register_post_accumulate_grad_hook(self._fold_grad(s)))
                else:
                    s.param.grad = self.grad[s.offset : s.offset + s.numel].view_as(s.param)
                if r != s.numel:
                    cols = s.param.shape[1]
                    s.param._bpe_padded = self.data[s.offset : s.offset + r].view(r // cols, cols)
                    s.param._bpe_padded_grad = self.grad[s.offset : s.offset + r].view(r // cols, cols)

    def _fold_grad(self, slot: Slot):
        dst = self.grad[slot.offset : slot.offset + slot.numel]

        def hook(p: Tensor) -> None:
            if p.grad is not None:
                with torch.no_grad():
                    dst.add_(p.grad.reshape(-1))
                p.grad = None

        return hook

    @classmethod
    def from_module(cls, module: nn.Module, grad_dtype: torch.dtype | None = None,
                    pad_to: int = ALIGN) -> "FlatParameters":
        for m in module.modules():  # row padding requested on the module (survives deepcopy / .to())
            rows = getattr(m, "pad_rows", None)
            if rows and isinstance(getattr(m, "weight", None), nn.Parameter):
                m.weight._bpe_pad_rows = rows
        return cls([(n, p) for n, p in module.named_parameters() if p.requires_grad], grad_dtype, pad_to)

    def zero_grad(self) -> None:
        self.grad.zero_()
        if self.split_grad:
            return
        for s in self.slots:  # re-attach in case someone set .grad = None
            if s.param.grad is None or s.param.grad.data_ptr() != self.grad[s.offset :].data_ptr():
                s.param.grad = self.grad[s.offset : s.offset + s.numel].view_as(s.param)

    def grad_view(self, slot: Slot) -> Tensor:
        return self.grad[slot.offset : slot.offset + slot.numel]


class FlatAdamW:
    """AdamW over a :class:`FlatParameters` with fp32 master weights and moments.

    Weight decay is applied to params with ``ndim >= 2`` by default (norm gains
    are not decayed); set ``decay_all=True`` for uniform decay.  On the GPU one
    kernel launch covers the whole buffer (a per-64-element decay mask); on the
    CPU, consecutive params with the same decay form one update each.

    The number of APPLIED updates lives on the device (``self.nstep``): a step
    whose gradient norm is non-finite is skipped by the kernels and does not
    advance it, so the bias correction and the checkpointed ``step`` count
    only real updates.  ``calls`` counts :meth:`step` invocations on the host.
    """

    def __init__(self, flat: FlatParameters, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01, decay_all: bool = False):
        self.flat = flat
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.decay_all = decay_all
        self.calls = 0
        self.nstep = torch.zeros(1, dtype=torch.int32, device=flat.device)
        self.master = flat.data.float() if flat.dtype != torch.float32 else flat.data
        self.exp_avg = torch.zeros(flat.numel, dtype=torch.float32, device=flat.device)
        self.exp_avg_sq = torch.zeros(flat.numel, dtype=torch.float32, device=flat.device)
        self.weight_decay = weight_decay
        self.shard: list[tuple[int, int]] | None = None  # element ranges this rank updates (ZeRO-1), None = all
        self._build_segments()

    def set_shard(self, ranges: list[tuple[int, int]] | None) -> None:
        """Restrict :meth:`step` to the element ranges ``[s, e)`` this rank owns (sharded data parallelism,
        ``parallel/zero.py``).  The moments and master weights stay full-size buffers -- at 288 GB of HBM the
        point of sharding is the optimizer's time and HBM traffic, not capacity -- but only the owned ranges are
        current; ``ShardedDataParallel.gather_optimizer_state`` makes all of them current on every rank (checkpoints)."""
        self.shard = sorted(ranges) if ranges is not None else None
        self._build_segments()

    def _build_segments(self) -> None:
        """Contiguous runs of equal weight decay, from ``self.weight_decay``; on the GPU also the per-64-element
        decay mask that lets one launch per owned range cover all of them (``wd_mask``)."""
        flat = self.flat
        self.segments: list[tuple[int, int, float]] = []
        for i, s in enumerate(flat.slots):
            wd = self.weight_decay if (self.decay_all or s.param.dim() >= 2) else 0.0
            end = flat.slots[i + 1].offset if i + 1 < len(flat.slots) else flat.numel
            if self.segments and self.segments[-1][2] == wd and self.segments[-1][1] == s.offset:
                self.segments[-1] = (self.segments[-1][0], end, wd)
            else:
                self.segments.append((s.offset, end, wd))
        # one byte per 64 elements (slots are 64-aligned): 1 where the segment decays.  With one decay value the
        # mask lets a single launch per owned range replace the per-segment launches (27 at GPT-2-small)
        self.wd_mask = None
        wds = {wd for _, _, wd in self.segments}
        if flat.device.type == "cuda" and len(wds - {0.0}) <= 1 and all(a % 64 == 0 for a, _, _ in self.segments):
            mask = torch.zeros((flat.numel + 63) // 64, dtype=torch.uint8)
            for a, b, wd in self.segments:
                if wd != 0.0:
                    mask[a // 64 : (b + 63) // 64] = 1
            self.wd_mask = mask.to(flat.device)
            self.mask_wd = next(iter(wds - {0.0}), 0.0)
        if self.shard is not None:  # intersect with the owned ranges: one launch per (segment, range) overlap
            self.segments = [(max(a, s), min(b, e), wd) for a, b, wd in self.segments for s, e in self.shard
                             if max(a, s) < min(b, e)]

    @property
    def step_count(self) -> int:
        """Updates actually applied (reads the device counter: a host sync)."""
        return int(self.nstep.item())

    @torch.no_grad()
    def clip_grad_norm(self, max_norm: float) -> tuple[Tensor, Tensor]:
        """Returns (norm, coef) as device scalars; the coef is applied inside :meth:`step`."""
        return grad_norm([self.flat.grad], max_norm)

    @torch.no_grad()
    def step(self, lr: float | None = None, grad_scale: Tensor | None = None) -> None:
        if lr is not None:
            self.lr = lr
        self.calls += 1
        b1, b2 = self.betas
        out = self.flat.data if self.flat.dtype == torch.bfloat16 else None
        count_adam_step(self.nstep, grad_scale)
        if self.wd_mask is not None and all(s % 64 == 0 for s, _ in (self.shard or [(0, 0)])):
            for s, e in (self.shard or [(0, self.flat.numel)]):  # one launch per owned range
                fused_adamw_step(
                    self.master[s:e], self.exp_avg[s:e], self.exp_avg_sq[s:e], self.flat.grad[s:e],
                    out[s:e] if out is not None else None, self.lr, b1, b2, self.eps, self.mask_wd, 0, grad_scale,
                    self.nstep, self.wd_mask[s // 64 :],
                )
        else:
            for s, e, wd in self.segments:
                fused_adamw_step(
                    self.master[s:e], self.exp_avg[s:e], self.exp_avg_sq[s:e], self.flat.grad[s:e],
                    out[s:e] if out is not None else None, self.lr, b1, b2, self.eps, wd, 0, grad_scale, self.nstep,
                )
        if out is None and self.master is not self.flat.data:
            for s, e in (self.shard or [(0, self.flat.numel)]):
                self.flat.data[s:e].copy_(self.master[s:e])

    def state_dict(self) -> dict:
        """The flat buffers are saved up to the end of the last parameter (``flat.used``), not with the zero tail
        that the sharding pad (``pad_to = world x 64``) adds, so a checkpoint resumes on any world size and with
        or without ZeRO-1."""
        u = self.flat.used
        return {
            "step": self.step_count, "lr": self.lr, "betas": tuple(self.betas), "eps": self.eps,
            "weight_decay": self.weight_decay, "master": self.master[:u], "exp_avg": self.exp_avg[:u],
            "exp_avg_sq": self.exp_avg_sq[:u],
        }

    @torch.no_grad()
    def load_state_dict(self, sd: dict) -> None:
        self.nstep.fill_(int(sd["step"]))
        self.lr = float(sd["lr"])
        self.betas = tuple(sd["betas"])
        self.eps = float(sd["eps"])
        self.weight_decay = float(sd["weight_decay"])
        self._build_segments()  # the per-segment decay follows the restored value
        for name, buf in (("master", self.master), ("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
            src = sd[name].reshape(-1)
            n = min(src.numel(), buf.numel())
            if src.numel() < self.flat.used:
                raise ValueError(f"optimizer state '{name}' has {src.numel()} elements, the model needs "
                                 f"{self.flat.used}")
            buf[:n].copy_(src[:n])  # older checkpoints may carry a padded tail: only the zero pad differs
            buf[n:].zero_()
        if self.master is not self.flat.data:
            self.flat.data.copy_(self.master)
