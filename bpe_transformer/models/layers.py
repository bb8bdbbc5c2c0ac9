"""Transformer building blocks.

State-dict keys and weight shapes follow the reference contract exactly
(``tests/adapters.py:209-361``): ``attn.{q,k,v,output}_proj.weight``,
``ln1.weight``, ``ffn.{w1,w2,w3}.weight``, ``ln2.weight``,
``token_embeddings.weight``, ``ln_final.weight``, ``lm_head.weight``; all
linear weights are PyTorch-style ``(d_out, d_in)``.

Two execution paths share these modules:
  * CPU / fp32 / arbitrary masks: the oracle ops of ``models.functional``.
  * GPU bf16 (the training hot path): hipBLASLt GEMMs for the projections and
    the gfx950 HIP kernels of ``bpe_transformer.ops`` for everything else, with
    these fusions: one [Wq;Wk;Wv] GEMM -> flash attention with RoPE applied
    inside the kernel -> output projection with the residual add folded into
    the GEMM (addmm); one [W1;W3] GEMM -> SwiGLU gate kernel -> W2 GEMM + residual.
"""

from __future__ import annotations

import math

import torch
from torch import Tensor, nn

from .. import ops
from . import functional as F


def _trunc_normal_(w: Tensor, std: float) -> Tensor:
    return nn.init.trunc_normal_(w, mean=0.0, std=std, a=-3 * std, b=3 * std)


class Linear(nn.Module):
    """Bias-free linear layer, ``y = x @ W^T`` with ``W: (d_out, d_in)`` (contract K1)."""

    def __init__(self, in_features: int, out_features: int, device=None, dtype=None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, device=device, dtype=dtype))
        _trunc_normal_(self.weight, math.sqrt(2.0 / (in_features + out_features)))

    def forward(self, x: Tensor) -> Tensor:
        return torch.matmul(x, self.weight.t())

    def extra_repr(self) -> str:
        return f"in_features={self.in_features}, out_features={self.out_features}"


class Embedding(nn.Module):
    """Token embedding lookup ``W[ids]`` with ``W: (num_embeddings, embedding_dim)`` (contract K2)."""

    def __init__(self, num_embeddings: int, embedding_dim: int, device=None, dtype=None):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.weight = nn.Parameter(torch.empty(num_embeddings, embedding_dim, device=device, dtype=dtype))
        _trunc_normal_(self.weight, 1.0)

    def forward(self, token_ids: Tensor) -> Tensor:
        return ops.embedding(self.weight, token_ids)


class RMSNorm(nn.Module):
    """RMSNorm with fp32 statistics (contract K4)."""

    def __init__(self, d_model: int, eps: float = 1e-5, device=None, dtype=None):
        super().__init__()
        self.d_model = d_model
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d_model, device=device, dtype=dtype))

    def forward(self, x: Tensor) -> Tensor:
        return ops.rmsnorm(x, self.weight, self.eps)


class RotaryPositionalEmbedding(nn.Module):
    """Interleaved RoPE with precomputed fp32 cos/sin tables ``[max_seq_len, d_k/2]`` (contract K8)."""

    def __init__(self, theta: float, d_k: int, max_seq_len: int, device=None):
        super().__init__()
        self.theta = theta
        self.d_k = d_k
        self.max_seq_len = max_seq_len
        cos, sin = F.rope_tables(d_k, max_seq_len, theta, device=device)
        self.register_buffer("cos", cos, persistent=False)
        self.register_buffer("sin", sin, persistent=False)

    def _apply(self, fn, recurse=True):
        # keep the tables fp32 when the module is cast to bf16
        cos, sin = self.cos, self.sin
        super()._apply(fn, recurse)
        self.cos = cos.to(self.cos.device)
        self.sin = sin.to(self.sin.device)
        return self

    def forward(self, x: Tensor, token_positions: Tensor | None = None) -> Tensor:
        return ops.apply_rope(x, self.cos, self.sin, token_positions)


class SwiGLU(nn.Module):
    """``W2(SiLU(W1 x) * W3 x)`` (contract K5)."""

    def __init__(self, d_model: int, d_ff: int, device=None, dtype=None):
        super().__init__()
        # registration order w1, w3, w2 keeps [W1; W3] adjacent in the flat parameter buffer
        self.w1 = Linear(d_model, d_ff, device=device, dtype=dtype)
        self.w3 = Linear(d_model, d_ff, device=device, dtype=dtype)
        self.w2 = Linear(d_ff, d_model, device=device, dtype=dtype)

    def fused_gate_up(self, x2: Tensor) -> Tensor:
        gu = torch.matmul(x2, torch.cat([self.w1.weight, self.w3.weight], 0).t())
        return ops.swiglu_gate(gu)

    def forward(self, x: Tensor) -> Tensor:
        if x.is_cuda:
            shp = x.shape
            a = self.fused_gate_up(x.reshape(-1, shp[-1]))
            return self.w2(a).view(*shp[:-1], -1)
        return self.w2(F.silu(self.w1(x)) * self.w3(x))


class ActFFN(nn.Module):
    """Two-matrix FFN ``W2(act(W1 x))`` for the ``ffn_type`` ablations ("silu", "gelu")."""

    def __init__(self, d_model: int, d_ff: int, act: str = "silu", device=None, dtype=None):
        super().__init__()
        self.act = act
        self.w1 = Linear(d_model, d_ff, device=device, dtype=dtype)
        self.w2 = Linear(d_ff, d_model, device=device, dtype=dtype)

    def forward(self, x: Tensor) -> Tensor:
        h = self.w1(x)
        h = ops.gelu(h) if self.act == "gelu" else ops.silu(h)
        return self.w2(h)


class MultiHeadSelfAttention(nn.Module):
    """Causal multi-head self-attention, optional RoPE and grouped KV heads (contracts K9, K10).

    ``q_proj`` rows are the heads concatenated (``(num_heads * d_k, d_model)``).
    """

    def __init__(
        self,
        d_model: int,
        num_heads: int,
        max_seq_len: int | None = None,
        theta: float | None = None,
        use_rope: bool = True,
        num_kv_heads: int | None = None,
        device=None,
        dtype=None,
    ):
        super().__init__()
        assert d_model % num_heads == 0, "d_model must be divisible by num_heads"
        self.d_model = d_model
        self.num_heads = num_heads
        self.num_kv_heads = num_kv_heads or num_heads
        assert num_heads % self.num_kv_heads == 0
        self.d_k = d_model // num_heads
        kv = self.num_kv_heads * self.d_k
        self.q_proj = Linear(d_model, d_model, device=device, dtype=dtype)
        self.k_proj = Linear(d_model, kv, device=device, dtype=dtype)
        self.v_proj = Linear(d_model, kv, device=device, dtype=dtype)
        self.output_proj = Linear(d_model, d_model, device=device, dtype=dtype)
        self.rope = None
        if use_rope and theta is not None and max_seq_len is not None:
            self.rope = RotaryPositionalEmbedding(theta, self.d_k, max_seq_len, device=device)

    def qkv_weight(self) -> Tensor:
        return torch.cat([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight], 0)

    def _fused_ok(self, x: Tensor, token_positions) -> bool:
        return (
            token_positions is None
            and x.dim() == 3
            and ops.flash_supported(x, self.d_k)
            and (self.rope is None or x.shape[1] <= self.rope.max_seq_len)
        )

    def attend(self, x2: Tensor, batch: int, seq: int) -> Tensor:
        """Fused GPU path on ``x2 = [batch*seq, d_model]``; returns pre-output-projection ``[batch*seq, d_model]``."""
        qkv = torch.matmul(x2, self.qkv_weight().t())
        cos = self.rope.cos if self.rope is not None else None
        sin = self.rope.sin if self.rope is not None else None
        return ops.flash_attention_qkv(qkv, batch, seq, self.num_heads, self.num_kv_heads, self.d_k, cos, sin, True)

    def forward(self, x: Tensor, token_positions: Tensor | None = None) -> Tensor:
        if self._fused_ok(x, token_positions):
            B, S, _ = x.shape
            o = self.attend(x.reshape(B * S, -1), B, S)
            return self.output_proj(o).view(B, S, -1)
        return self._forward_reference(x, token_positions)

    def _forward_reference(self, x: Tensor, token_positions: Tensor | None) -> Tensor:
        *lead, S, _ = x.shape
        H, Hkv, D = self.num_heads, self.num_kv_heads, self.d_k
        q = self.q_proj(x).view(*lead, S, H, D).transpose(-2, -3)
        k = self.k_proj(x).view(*lead, S, Hkv, D).transpose(-2, -3)
        v = self.v_proj(x).view(*lead, S, Hkv, D).transpose(-2, -3)
        if self.rope is not None:
            pos = token_positions
            if pos is not None and pos.dim() >= 2:
                pos = pos.unsqueeze(-2)  # [..., S] -> [..., 1(head), S]
            q = self.rope(q, pos)
            k = self.rope(k, pos)
        if Hkv != H:
            k = k.repeat_interleave(H // Hkv, dim=-3)
            v = v.repeat_interleave(H // Hkv, dim=-3)
        mask = F.causal_mask(S, device=x.device)
        o = F.scaled_dot_product_attention(q, k, v, mask)
        o = o.transpose(-2, -3).reshape(*lead, S, H * D)
        return self.output_proj(o)


class TransformerBlock(nn.Module):
    """Pre-norm block ``h = x + MHA(RMSNorm1(x)); y = h + FFN(RMSNorm2(h))`` (contract K11).

    Ablations from the reference's ``model_config.json`` schema: ``remove_rmsnorm``,
    ``use_post_norm``, ``remove_rope``, ``ffn_type`` in {None/"swiglu", "silu", "gelu"}.
    """

    def __init__(
        self,
        d_model: int,
        num_heads: int,
        d_ff: int,
        max_seq_len: int,
        theta: float = 10000.0,
        num_kv_heads: int | None = None,
        remove_rmsnorm: bool = False,
        use_post_norm: bool = False,
        remove_rope: bool = False,
        ffn_type: str | None = None,
        eps: float = 1e-5,
        device=None,
        dtype=None,
    ):
        super().__init__()
        self.remove_rmsnorm = remove_rmsnorm
        self.use_post_norm = use_post_norm
        self.attn = MultiHeadSelfAttention(
            d_model, num_heads, max_seq_len, theta, use_rope=not remove_rope, num_kv_heads=num_kv_heads,
            device=device, dtype=dtype,
        )
        self.ln1 = RMSNorm(d_model, eps, device=device, dtype=dtype) if not remove_rmsnorm else nn.Identity()
        self.ln2 = RMSNorm(d_model, eps, device=device, dtype=dtype) if not remove_rmsnorm else nn.Identity()
        ffn_type = (ffn_type or "swiglu").lower()
        self.ffn_type = ffn_type
        if ffn_type == "swiglu":
            self.ffn = SwiGLU(d_model, d_ff, device=device, dtype=dtype)
        elif ffn_type in ("silu", "gelu"):
            self.ffn = ActFFN(d_model, d_ff, ffn_type, device=device, dtype=dtype)
        else:
            raise ValueError(f"unknown ffn_type {ffn_type!r}")

    def _fused_ok(self, x: Tensor) -> bool:
        return (
            not self.use_post_norm
            and not self.remove_rmsnorm
            and self.ffn_type == "swiglu"
            and self.attn._fused_ok(x, None)
        )

    def forward(self, x: Tensor, token_positions: Tensor | None = None) -> Tensor:
        if token_positions is None and self._fused_ok(x):
            return self._forward_fused(x)
        if self.use_post_norm:
            x = self.ln1(x + self.attn(x, token_positions))
            return self.ln2(x + self.ffn(x))
        x = x + self.attn(self.ln1(x), token_positions)
        return x + self.ffn(self.ln2(x))

    def _forward_fused(self, x: Tensor) -> Tensor:
        from .fused_block import fused_block_forward

        return fused_block_forward(self, x)

    def _forward_fused_unfused_ops(self, x: Tensor) -> Tensor:
        """Same math as :meth:`_forward_fused` through per-op autograd (kept for A/B and debugging)."""
        B, S, d = x.shape
        x2 = x.reshape(B * S, d)
        o = self.attn.attend(self.ln1(x2), B, S)
        x2 = torch.addmm(x2, o, self.attn.output_proj.weight.t())  # residual folded into the GEMM
        a = self.ffn.fused_gate_up(self.ln2(x2))
        x2 = torch.addmm(x2, a, self.ffn.w2.weight.t())
        return x2.view(B, S, d)
