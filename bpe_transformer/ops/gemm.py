"""Hand-written gfx950 split-K MFMA GEMM (``csrc/gemm.hip``) for weight gradients.

``accumulate_weight_grad(g, dy, x)`` computes ``g += dy^T @ x`` where
``dy: [T, N]`` and ``x: [T, K]`` are token-major activations (T = batch*seq)
and ``g: [N, K]`` is a view of the flat bf16 gradient buffer.  The reduction
runs over all T tokens, which for a training step is large (16k-64k) while
N x K is small: the kernel splits T across workgroups (enough to fill all 256
CUs) and reduces the fp32 partials deterministically into ``g``.  Shapes the
kernel does not cover (N or K not a multiple of 128, T not a multiple of
64 * splits) go to hipBLASLt (``addmm_``).
"""

from __future__ import annotations

import os

import torch
from torch import Tensor

from ._ext import ops

_TARGET_WGS = int(os.environ.get("BPE_GEMM_TARGET_WGS", "512"))
_ENABLED = os.environ.get("BPE_DW_GEMM", "1") == "1"


def choose_splits(n: int, k: int, t: int, target: int = _TARGET_WGS, min_iters: int = 8) -> int:
    tiles = (n // 128) * (k // 128)
    best = 1
    s = 1
    while s <= 64:
        if t % (64 * s) == 0 and t // (64 * s) >= min_iters:
            best = s
            if tiles * s >= target:
                break
        s *= 2
    return best


_MAX_TILES = int(os.environ.get("BPE_DW_GEMM_MAX_TILES", "160"))


def supported(n: int, k: int, t: int) -> bool:
    """Shapes routed to the split-K kernel: tile-aligned and with few output tiles.

    Measured on MI355X (benchmarks/gemm_bench.py, 16k and 64k tokens): the split-K kernel beats hipBLASLt
    1.25-1.67x on the 768x768 / 2304x768 / 768x2048 gradients (36-108 tiles of 128x128) and loses ~10% on
    the 4096x768 one (192 tiles), where the library's own tiles already fill the chip.
    """
    return n % 128 == 0 and k % 128 == 0 and t % 64 == 0 and (n // 128) * (k // 128) <= _MAX_TILES


def accumulate_weight_grad(g: Tensor, dy: Tensor, x: Tensor) -> None:
    """``g += dy.T @ x`` (bf16, fp32 accumulation)."""
    n, k = g.shape
    t = dy.shape[0]
    if (_ENABLED and g.is_cuda and g.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16
            and x.dtype == torch.bfloat16 and supported(n, k, t) and g.stride(1) == 1 and dy.stride(1) == 1
            and x.stride(1) == 1):
        ops().gemm(dy, False, x, False, g, 1.0, choose_splits(n, k, t))
    else:
        g.addmm_(dy.t(), x)


def matmul_nt(a: Tensor, b: Tensor, out: Tensor | None = None, beta: float = 0.0) -> Tensor:
    """``out = beta*out + a @ b.T`` with a: [M, R], b: [N, R] (both K-major) on the HIP kernel."""
    m, r = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty(m, n, device=a.device, dtype=a.dtype)
        beta = 0.0
    ops().gemm(a, True, b, True, out, beta, choose_splits(m, n, r))
    return out
