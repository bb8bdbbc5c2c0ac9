"""RMSNorm op: HIP kernel on the GPU, oracle on the CPU.

Reference contract K4 (``tests/adapters.py:364-384`` in the reference).
"""

from __future__ import annotations

import torch
from torch import Tensor

from . import reference as F
from ._ext import ops


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, w: Tensor, eps: float):
        y, rstd = ops().rmsnorm_fwd(x.contiguous(), w.contiguous(), eps)
        ctx.save_for_backward(x, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy: Tensor):
        x, w, rstd = ctx.saved_tensors
        dx, dw = ops().rmsnorm_bwd(dy, x.contiguous(), w.contiguous(), rstd)
        return dx, dw, None


def rmsnorm(x: Tensor, weight: Tensor, eps: float = 1e-5) -> Tensor:
    if x.is_cuda:
        if weight.dtype != x.dtype:
            weight = weight.to(x.dtype)
        return _RMSNormFn.apply(x, weight, eps)
    return F.rmsnorm(x, weight, eps)
