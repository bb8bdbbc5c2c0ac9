"""Standalone softmax op (``csrc/softmax.hip``); contract K6 (``tests/adapters.py:424``)."""

from __future__ import annotations

import torch
from torch import Tensor

from . import reference as F
from ._ext import ops


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor):
        y = ops().softmax_fwd(x)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy: Tensor):
        (y,) = ctx.saved_tensors
        return ops().softmax_bwd(dy, y)


def softmax(x: Tensor, dim: int = -1) -> Tensor:
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.numel() > 0:
        nd = x.dim()
        dim = dim % nd
        if dim == nd - 1:
            return _SoftmaxFn.apply(x)
        return _SoftmaxFn.apply(x.movedim(dim, -1)).movedim(-1, dim)
    return F.softmax(x, dim)
