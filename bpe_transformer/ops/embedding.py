"""Embedding gather / deterministic scatter-add (``csrc/embedding.hip``).

Reference contract K2 (``tests/adapters.py:38-57``).
"""

from __future__ import annotations

import torch
from torch import Tensor

from ._ext import ops


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight: Tensor, ids: Tensor):
        ids = ids.long().contiguous()
        ctx.save_for_backward(ids)
        ctx.vocab = weight.shape[0]
        return ops().embed_fwd(weight, ids)

    @staticmethod
    def backward(ctx, dout: Tensor):
        (ids,) = ctx.saved_tensors
        return ops().embed_bwd(dout, ids, ctx.vocab), None


def embedding(weight: Tensor, ids: Tensor) -> Tensor:
    if weight.is_cuda and weight.dtype in (torch.float32, torch.bfloat16) and (
        weight.shape[1] * weight.element_size()
    ) % 16 == 0:
        return _EmbeddingFn.apply(weight, ids)
    return weight[ids]
