"""FFN activation ops (SwiGLU gate, SiLU, tanh-GELU).

GPU: HIP kernels in ``csrc/activations.hip``.  CPU: oracle definitions.
Reference contracts K3 / K5 (``tests/adapters.py:60-89, 387-398``) and the
reference's Triton GELU (``bpe_transformer/kernels/triton/gelu.py:18-64``),
which here also gets a backward.
"""

from __future__ import annotations

import torch
from torch import Tensor

from . import reference as F
from ._ext import ops

SILU, GELU = 0, 1


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu: Tensor):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return ops().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, d: Tensor):
        (gu,) = ctx.saved_tensors
        return ops().swiglu_bwd(d, gu)


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, kind: int):
        x = x.contiguous()
        ctx.save_for_backward(x)
        ctx.kind = kind
        return ops().act_fwd(x, kind)

    @staticmethod
    def backward(ctx, d: Tensor):
        (x,) = ctx.saved_tensors
        return ops().act_bwd(d, x, ctx.kind), None


def swiglu_gate(gu: Tensor) -> Tensor:
    """``silu(gu[..., :F]) * gu[..., F:]`` for the fused [W1; W3] projection output."""
    if gu.is_cuda:
        return _SwiGLUFn.apply(gu)
    f = gu.shape[-1] // 2
    return F.silu(gu[..., :f]) * gu[..., f:]


def _vec_ok(x: Tensor) -> bool:
    return x.numel() % (8 if x.dtype == torch.bfloat16 else 4) == 0 and x.dtype in (torch.float32, torch.bfloat16)


def silu(x: Tensor) -> Tensor:
    if x.is_cuda and _vec_ok(x):
        return _ActFn.apply(x, SILU)
    return F.silu(x)


def gelu(x: Tensor) -> Tensor:
    """tanh-approximate GELU (the reference's ``kernels/triton/gelu.py`` op)."""
    if x.is_cuda and _vec_ok(x):
        return _ActFn.apply(x, GELU)
    return F.gelu_tanh(x)
