"""Optimizer-side kernels: fused AdamW update and global-L2-norm clipping.

Reference contracts K14 (clip, ``tests/adapters.py:458-467``) and K15 (AdamW,
``adapters.py:470-474``).  On the GPU the clip coefficient stays on the
device and is consumed by the AdamW kernel, so clip + step never sync the host.
"""

from __future__ import annotations

from collections.abc import Iterable

import torch
from torch import Tensor

from ._ext import ops


def grad_norm(tensors: list[Tensor], max_norm: float = float("inf")) -> tuple[Tensor, Tensor]:
    """Global L2 norm of ``tensors`` and the clip coefficient ``min(1, max/(norm+1e-6))``.

    Both results are 0-dim fp32 tensors on the tensors' device.
    """
    if tensors and tensors[0].is_cuda:
        ts = [t.contiguous() for t in tensors]
        return ops().grad_norm(ts, float(max_norm))
    if not tensors:
        z = torch.zeros(())
        return z, torch.ones(())
    total = torch.sqrt(sum((t.detach().float() ** 2).sum() for t in tensors))
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    coef = torch.where(torch.isfinite(total), coef, torch.full_like(coef, -1.0))  # -1: skip-step sentinel
    return total, coef


@torch.no_grad()
def clip_grad_norm_(parameters: Iterable[torch.nn.Parameter], max_l2_norm: float) -> Tensor:
    """In-place global-norm gradient clipping; params with ``grad is None`` are skipped.

    Matches ``torch.nn.utils.clip_grad_norm_`` (scale = max/(norm + 1e-6) when norm > max).
    Returns the pre-clip total norm.
    """
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.zeros(())
    norm, coef = grad_norm(grads, max_l2_norm)
    if grads[0].is_cuda:
        for g in grads:
            if g.is_contiguous():
                ops().scale_(g, coef)
            else:
                g.mul_(coef.to(g.dtype))
    elif bool(coef >= 0):  # coef -1 marks a non-finite norm: leave the gradients as they are
        for g in grads:
            g.mul_(coef.to(g.dtype))
    return norm


def fused_adamw_step(
    param_fp32: Tensor,
    exp_avg: Tensor,
    exp_avg_sq: Tensor,
    grad: Tensor,
    param_bf16_out: Tensor | None,
    lr: float,
    beta1: float,
    beta2: float,
    eps: float,
    weight_decay: float,
    step: int,
    grad_scale: Tensor | None = None,
    nstep: Tensor | None = None,
    wd_mask: Tensor | None = None,
) -> None:
    """One AdamW step over flat fp32 buffers (one kernel launch on the GPU).

    ``grad`` may be fp32 or bf16; ``param_bf16_out`` (optional) receives the
    bf16 copy of the updated fp32 master weights; ``grad_scale`` (optional
    0-dim fp32 device tensor) multiplies the gradient first (clip coefficient).
    ``nstep`` (optional one-element int32 tensor, see :func:`count_adam_step`)
    is the number of updates applied so far INCLUDING this one; when given,
    the bias correction is computed from it (on the device) and ``step`` is
    ignored, so skipped non-finite steps do not shift bc1/bc2.  ``wd_mask``
    (optional uint8, one byte per 64 elements) applies ``weight_decay`` only
    where it is nonzero: a flat buffer's decay and no-decay segments in one
    launch.
    """
    if nstep is not None and not param_fp32.is_cuda:
        step = int(nstep.item())
    bc1 = 1.0 - beta1**step
    bc2_sqrt = (1.0 - beta2**step) ** 0.5
    if param_fp32.is_cuda:
        ops().adamw_step(param_fp32, exp_avg, exp_avg_sq, grad, param_bf16_out, lr, beta1, beta2, eps, weight_decay,
                         bc1, bc2_sqrt, grad_scale, nstep, wd_mask)
        return
    if wd_mask is not None:  # per-64-element decay on the CPU path: expand the mask
        wdv = torch.repeat_interleave(wd_mask.to(torch.float32), 64)[: param_fp32.numel()] * weight_decay
    else:
        wdv = None
    g = grad.float()
    if grad_scale is not None:
        if not bool(grad_scale >= 0):  # non-finite grad norm: skip (same rule as the kernel)
            return
        g = g * grad_scale
    if wdv is not None:
        param_fp32.mul_(1.0 - lr * wdv)
    else:
        param_fp32.mul_(1.0 - lr * weight_decay)
    exp_avg.mul_(beta1).add_(g, alpha=1.0 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    denom = (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
    param_fp32.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if param_bf16_out is not None:
        param_bf16_out.copy_(param_fp32)


def count_adam_step(nstep: Tensor, grad_scale: Tensor | None = None) -> None:
    """``nstep += 1`` unless ``grad_scale`` is the non-finite-norm sentinel (-1); on the device, no host sync.

    Run once per optimizer step before the :func:`fused_adamw_step` launches that read ``nstep``.
    """
    if nstep.is_cuda:
        ops().adam_count_step(nstep, grad_scale)
    elif grad_scale is None or bool(grad_scale >= 0):
        nstep.add_(1)
