"""Standalone rotary positional embedding (``csrc/rope.hip``).

In the model hot path RoPE is fused into attention (``ops.attention``); this op
serves the standalone contract K8 (``tests/adapters.py:187-206``) and
attention calls with custom ``token_positions``.
"""

from __future__ import annotations

import torch
from torch import Tensor

from . import reference as F
from ._ext import ops


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x3: Tensor, pos: Tensor, cos: Tensor, sin: Tensor):
        ctx.save_for_backward(pos, cos, sin)
        return ops().rope(x3, pos, cos, sin, False)

    @staticmethod
    def backward(ctx, d: Tensor):
        pos, cos, sin = ctx.saved_tensors
        return ops().rope(d.contiguous(), pos, cos, sin, True), None, None, None


def apply_rope(x: Tensor, cos: Tensor, sin: Tensor, token_positions: Tensor | None = None) -> Tensor:
    """Rotate interleaved pairs of ``x[..., seq, d]`` at ``token_positions`` (default ``arange(seq)``)."""
    d = x.shape[-1]
    vec = 8 if x.dtype == torch.bfloat16 else 4
    if not (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and d % vec == 0):
        return F.apply_rope(x, cos, sin, token_positions)
    seq = x.shape[-2]
    if token_positions is None:
        token_positions = torch.arange(seq, device=x.device)
    pos = torch.broadcast_to(token_positions.to(x.device).long(), x.shape[:-1]).reshape(-1).contiguous()
    x3 = x.contiguous().view(-1, 1, d)
    y = _RopeFn.apply(x3, pos, cos.float().contiguous(), sin.float().contiguous())
    return y.view(x.shape)
