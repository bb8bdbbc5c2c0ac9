"""Attention ops.

``scaled_dot_product_attention``: the generic contract (K7, ``tests/adapters.py:92-110``) -- any leading dims, an
arbitrary boolean mask -- on ``csrc/masked_sdpa.hip`` for GPU tensors (fp32 math), the oracle on the CPU.

``flash_attention_qkv`` (the training path, ``csrc/flash_attn_*.hip``) consumes the output of the fused QKV projection
``[B*S, (H + 2*Hkv) * D]`` directly (no transposes, no separate RoPE pass) and
returns ``[B*S, H*D]`` ready for the output projection; its backward returns
the gradient in the same fused layout, feeding the QKV weight-gradient GEMM
directly.  Reference contracts K7/K9/K10 (``tests/adapters.py:92-184``).
"""

from __future__ import annotations

import math
import os

import torch
from torch import Tensor

from . import reference as F
from ._ext import ops

SUPPORTED_HEAD_DIMS = (64, 128)

_EMPTY: dict[torch.device, Tensor] = {}


def _empty(dev: torch.device) -> Tensor:
    t = _EMPTY.get(dev)
    if t is None:
        t = torch.empty(0, 0, device=dev, dtype=torch.float32)
        _EMPTY[dev] = t
    return t


class _MaskedSDPAFn(torch.autograd.Function):
    """Forward on the HIP kernel; the backward (not on the training path: the model's attention is the flash
    kernels') differentiates the oracle formula on the saved inputs."""

    @staticmethod
    def forward(ctx, q: Tensor, k: Tensor, v: Tensor, mask: Tensor | None, scale: float):
        ctx.save_for_backward(q, k, v, mask)
        ctx.scale = scale
        return ops().masked_sdpa(q, k, v, mask, scale)

    @staticmethod
    def backward(ctx, do: Tensor):
        q, k, v, mask = ctx.saved_tensors
        with torch.enable_grad():
            qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
            s = torch.matmul(qf, kf.transpose(-1, -2)) * ctx.scale
            if mask is not None:
                s = s.masked_fill(mask == 0, float("-inf"))
            o = torch.matmul(torch.softmax(s, -1), vf)
            dq, dk, dv = torch.autograd.grad(o, (qf, kf, vf), do.float())
        return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None, None


def scaled_dot_product_attention(Q: Tensor, K: Tensor, V: Tensor, mask: Tensor | None = None,
                                 scale: float | None = None) -> Tensor:
    """``softmax(Q K^T * scale + (mask ? 0 : -inf)) V`` (scale 1/sqrt(d_k) by default) with any leading dims and a
    boolean mask (True = attend; an integer 0/1 mask counts nonzero as attend) broadcastable to ``[..., q, k]``.
    A floating-point mask is refused: torch reads one as ADDITIVE (0 = attend, -inf = block), the opposite of the
    nonzero-means-attend reading, and the reference contract (``tests/adapters.py:96``) takes boolean masks only.
    GPU fp32 / bf16 tensors run ``csrc/masked_sdpa.hip`` (fp32 math, head dims up to 128, at most 65535 batch-heads);
    anything else the oracle formula (``ops.reference``, with the same mask semantics)."""
    d_k = Q.shape[-1]
    if mask is not None and mask.dtype != torch.bool:
        if mask.is_floating_point():
            raise TypeError("scaled_dot_product_attention: a floating-point mask is ambiguous (torch reads it as "
                            "additive); pass a boolean mask (True = attend)")
        mask = mask != 0  # 0/1 integer masks: nonzero = attend, on every path
    # the HIP kernel's grid.y is the batch-head count: at most 65535 (more falls back like other unsupported inputs)
    if not (Q.is_cuda and Q.dtype in (torch.float32, torch.bfloat16) and K.dtype == Q.dtype and V.dtype == Q.dtype
            and d_k <= 128 and V.shape[-1] <= 128 and Q.shape[:-2] == K.shape[:-2] == V.shape[:-2]
            and math.prod(Q.shape[:-2]) <= 65535):
        if scale is None:
            return F.scaled_dot_product_attention(Q, K, V, mask)
        s = torch.matmul(Q, K.transpose(-1, -2)) * scale
        if mask is not None:
            s = s.masked_fill(~mask, float("-inf"))
        return torch.matmul(F.softmax(s, -1), V)
    lead = Q.shape[:-2]
    Sq, Sk = Q.shape[-2], K.shape[-2]
    q, k, v = (t.reshape(-1, t.shape[-2], t.shape[-1]) for t in (Q, K, V))
    m = None
    if mask is not None:  # a view where the broadcast allows it (stride 0), else a copy
        m = mask.to(device=Q.device).expand(*lead, Sq, Sk).reshape(-1, Sq, Sk)
    o = _MaskedSDPAFn.apply(q, k, v, m, 1.0 / math.sqrt(d_k) if scale is None else scale)
    return o.reshape(*lead, Sq, V.shape[-1])


def prerotate_default(head_dim: int) -> bool:
    """Rotate Q / K once in the QKV activation instead of inside the attention kernels: the D = 64 forward (v8)
    then stages K by LDS-DMA with no per-tile rotation, and the split backward (D = 64 and 128) takes the pre-rotated
    operands as they are (at D = 128 the in-kernel form costs the backward a rotated copy: B 4 S 2048, forward +
    backward 0.505 vs 0.618 ms MHA, 0.877 vs 1.048 ms GQA 32:8, ``profiles/bench/attn_d128_split_r4.log``).  The fused
    blocks apply that rotation in the QKV GEMM's epilogue (``gemm_qkv_rope``; ``rope_qk_`` in place on the fp8 path
    and here, for a given qkv tensor).  ``BPE_ROPE_PREROTATE=0`` keeps the fused-RoPE attention kernels."""
    return head_dim in (64, 128) and os.environ.get("BPE_ROPE_PREROTATE", "1") == "1"


class _FlashAttnQKVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv: Tensor, cos, sin, B: int, S: int, H: int, Hkv: int, D: int, causal: bool, scale: float,
                prerotate: bool):
        use_rope = cos is not None
        c = cos if use_rope else _empty(qkv.device)
        s = sin if use_rope else _empty(qkv.device)
        pre = use_rope and prerotate
        if pre:  # rotate a copy (the input belongs to autograd); the backward re-reads the rotated copy
            qkv = qkv.clone()
            ops().rope_qk_(qkv, c, s, B, S, H, Hkv, D)
        q = qkv[:, : H * D]
        k = qkv[:, H * D : (H + Hkv) * D]
        v = qkv[:, (H + Hkv) * D :]
        o, lse = ops().fa_fwd(q, k, v, c, s, B, S, H, Hkv, D, causal, use_rope, scale, pre)
        ctx.save_for_backward(qkv, o, lse, c, s)
        ctx.meta = (B, S, H, Hkv, D, causal, use_rope, scale, pre)
        return o

    @staticmethod
    def backward(ctx, do: Tensor):
        qkv, o, lse, c, s = ctx.saved_tensors
        B, S, H, Hkv, D, causal, use_rope, scale, pre = ctx.meta
        q = qkv[:, : H * D]
        k = qkv[:, H * D : (H + Hkv) * D]
        v = qkv[:, (H + Hkv) * D :]
        dqkv = ops().fa_bwd(do, q, k, v, o, lse, c, s, B, S, H, Hkv, D, causal, use_rope, scale, pre)
        return dqkv, None, None, None, None, None, None, None, None, None, None


def flash_supported(x: Tensor, head_dim: int) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16 and head_dim in SUPPORTED_HEAD_DIMS


def flash_attention_qkv(
    qkv: Tensor,
    batch: int,
    seq: int,
    n_heads: int,
    n_kv_heads: int,
    head_dim: int,
    cos: Tensor | None = None,
    sin: Tensor | None = None,
    causal: bool = True,
    scale: float | None = None,
    prerotate: bool | None = None,
) -> Tensor:
    """Attention over a fused QKV activation.

    qkv: ``[batch*seq, (n_heads + 2*n_kv_heads) * head_dim]`` bf16 on the GPU.
    cos/sin: fp32 ``[>=seq, head_dim/2]`` RoPE tables (positions ``0..seq-1``),
    or ``None`` for no RoPE.  Returns ``[batch*seq, n_heads*head_dim]``.
    ``prerotate``: apply RoPE to a copy of Q / K first (``rope_qk_``) and run the
    kernels in pre-rotated mode (default :func:`prerotate_default`).
    """
    if prerotate is None:
        prerotate = prerotate_default(head_dim)
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    if qkv.is_cuda:
        if qkv.stride(1) != 1 or qkv.stride(0) % 8 != 0:
            qkv = qkv.contiguous()
        if cos is not None:
            cos = cos.float().contiguous()
            sin = sin.float().contiguous()
        return _FlashAttnQKVFn.apply(qkv, cos, sin, batch, seq, n_heads, n_kv_heads, head_dim, causal, scale,
                                     bool(prerotate))
    return attention_qkv_reference(qkv, batch, seq, n_heads, n_kv_heads, head_dim, cos, sin, causal, scale)


def attention_qkv_reference(qkv, batch, seq, n_heads, n_kv_heads, head_dim, cos=None, sin=None, causal=True,
                            scale=None) -> Tensor:
    """Oracle implementation of :func:`flash_attention_qkv` (fp32 math)."""
    H, Hkv, D = n_heads, n_kv_heads, head_dim
    x = qkv.float().view(batch, seq, H + 2 * Hkv, D)
    q = x[:, :, :H].transpose(1, 2)
    k = x[:, :, H : H + Hkv].transpose(1, 2)
    v = x[:, :, H + Hkv :].transpose(1, 2)
    if cos is not None:
        q = F.apply_rope(q, cos.float(), sin.float())
        k = F.apply_rope(k, cos.float(), sin.float())
    if Hkv != H:
        k = k.repeat_interleave(H // Hkv, dim=1)
        v = v.repeat_interleave(H // Hkv, dim=1)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(~F.causal_mask(seq, device=s.device), float("-inf"))
    o = torch.matmul(F.softmax(s, -1), v)
    return o.transpose(1, 2).reshape(batch * seq, H * D).to(qkv.dtype)
