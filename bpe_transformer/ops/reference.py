"""Reference ("oracle") functional ops in plain PyTorch.

These are the short, obviously-correct fp32 definitions every HIP kernel in
``bpe_transformer.ops`` is tested against, and the implementation used on CPU
(which is what the reference's adapter contract exercises,
``tests/adapters.py:16-542`` in the reference).

Conventions verified against the reference snapshots:
  * SDPA mask: ``True`` = attend, ``False`` -> ``-inf``; scale ``1/sqrt(d_k)``.
  * RoPE: *interleaved* pairs ``(x[2i], x[2i+1])``, ``inv_freq_i = theta^(-2i/d)``.
  * Cross-entropy: mean over rows of ``logsumexp(x) - x[target]``.
"""

from __future__ import annotations

import math

import torch
from torch import Tensor


def softmax(x: Tensor, dim: int = -1) -> Tensor:
    """Numerically stable softmax (reference contract ``adapters.py:424``)."""
    x_max = x.amax(dim=dim, keepdim=True)
    e = torch.exp(x - x_max)
    return e / e.sum(dim=dim, keepdim=True)


def log_softmax(x: Tensor, dim: int = -1) -> Tensor:
    x_max = x.amax(dim=dim, keepdim=True)
    z = x - x_max
    return z - torch.log(torch.exp(z).sum(dim=dim, keepdim=True))


def silu(x: Tensor) -> Tensor:
    """``x * sigmoid(x)`` (``adapters.py:387``)."""
    return x * torch.sigmoid(x)


def gelu_tanh(x: Tensor) -> Tensor:
    """tanh-approximate GELU, the op of the reference's only GPU kernel
    (``bpe_transformer/kernels/triton/gelu.py:33-64``).  Uses ``torch.tanh``,
    which saturates correctly; the reference's ``(e^{2a}-1)/(e^{2a}+1)`` form is
    NaN for large positive ``x``."""
    c = math.sqrt(2.0 / math.pi)
    return 0.5 * x * (1.0 + torch.tanh(c * (x + 0.044715 * x * x * x)))


def cross_entropy(logits: Tensor, targets: Tensor) -> Tensor:
    """Mean cross-entropy over all leading dims (``adapters.py:440``)."""
    logits = logits.reshape(-1, logits.shape[-1]).float()
    targets = targets.reshape(-1)
    m = logits.amax(dim=-1, keepdim=True)
    lse = (m + torch.log(torch.exp(logits - m).sum(dim=-1, keepdim=True))).squeeze(-1)
    tgt = logits.gather(-1, targets.unsqueeze(-1)).squeeze(-1)
    return (lse - tgt).mean()


def rmsnorm(x: Tensor, weight: Tensor, eps: float = 1e-5) -> Tensor:
    """RMSNorm with fp32 statistics (``adapters.py:364``)."""
    in_dtype = x.dtype
    xf = x.float()
    rms = torch.rsqrt(xf.pow(2).mean(dim=-1, keepdim=True) + eps)
    return (xf * rms * weight.float()).to(in_dtype)


def rope_tables(d_k: int, max_seq_len: int, theta: float, device=None) -> tuple[Tensor, Tensor]:
    """cos/sin tables of shape ``[max_seq_len, d_k // 2]`` (fp32)."""
    assert d_k % 2 == 0, "RoPE needs an even head dimension"
    inv_freq = theta ** (-torch.arange(0, d_k, 2, dtype=torch.float64, device=device) / d_k)
    pos = torch.arange(max_seq_len, dtype=torch.float64, device=device)
    ang = torch.outer(pos, inv_freq)
    return torch.cos(ang).float(), torch.sin(ang).float()


def apply_rope(x: Tensor, cos: Tensor, sin: Tensor, token_positions: Tensor | None = None) -> Tensor:
    """Rotate interleaved pairs of the last dim of ``x`` (``adapters.py:187``).

    ``cos``/``sin``: ``[max_seq_len, d/2]``.  ``token_positions`` broadcasts
    against ``x.shape[:-1]``; ``None`` means ``arange(seq_len)``.
    """
    seq = x.shape[-2]
    if token_positions is None:
        token_positions = torch.arange(seq, device=x.device)
    c = cos[token_positions].to(x.dtype)
    s = sin[token_positions].to(x.dtype)
    x1 = x[..., 0::2]
    x2 = x[..., 1::2]
    out = torch.empty_like(x)
    out[..., 0::2] = x1 * c - x2 * s
    out[..., 1::2] = x1 * s + x2 * c
    return out


def scaled_dot_product_attention(Q: Tensor, K: Tensor, V: Tensor, mask: Tensor | None = None) -> Tensor:
    """``softmax(QK^T/sqrt(d_k) + mask) V`` with arbitrary leading dims
    (``adapters.py:92``).  ``mask`` is boolean, True = keep."""
    d_k = Q.shape[-1]
    scores = torch.matmul(Q, K.transpose(-1, -2)) / math.sqrt(d_k)
    if mask is not None:
        scores = scores.masked_fill(~mask, float("-inf"))
    return torch.matmul(softmax(scores, dim=-1), V)


def causal_mask(seq_q: int, seq_k: int | None = None, device=None) -> Tensor:
    seq_k = seq_q if seq_k is None else seq_k
    return torch.ones(seq_q, seq_k, dtype=torch.bool, device=device).tril(diagonal=seq_k - seq_q)
