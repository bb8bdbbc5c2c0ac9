"""KV-cache ops of the serving path (``csrc/decode_attn.hip``).

The reference has no inference engine ("absent layers"); these ops
let ``models.generation`` decode with a KV cache instead of re-running the
whole prefix for every new token.

* :func:`kv_append` takes the fused QKV projection of ``T`` new tokens per
  sequence, applies RoPE at their absolute positions (``pos .. pos+T-1``, with
  ``pos`` a device int32 tensor), writes K (roped) and V into the caches
  ``[B, Hkv, Lmax, D]``, and returns the roped queries ``[B*T, H*D]``.
* :func:`decode_gemv` / :func:`decode_qkv` are the M <= 8 skinny projections of
  the decode step with RMSNorm / residual-add prologues and SwiGLU / RoPE +
  cache-write epilogues (``csrc/decode_gemv.hip``).
* :func:`decode_attention` is single-token attention of ``q [B, H*D]`` over the
  first ``pos + 1`` cache rows (split-K "flash-decoding" with a combine pass).

Both read the position from device memory, so a decode step is shape-static and
can be captured in a HIP graph.  The CPU versions are the oracle.
"""

from __future__ import annotations

import math

import torch
from torch import Tensor

from . import reference as F
from ._ext import ops


def kv_append(qkv: Tensor, k_cache: Tensor, v_cache: Tensor, cos: Tensor | None, sin: Tensor | None, pos: Tensor,
              batch: int, n_new: int, n_heads: int) -> Tensor:
    if qkv.is_cuda:
        use_rope = cos is not None
        c = cos if use_rope else qkv.new_empty(0, dtype=torch.float32)
        s = sin if use_rope else qkv.new_empty(0, dtype=torch.float32)
        return ops().kv_append(qkv, k_cache, v_cache, c, s, pos, batch, n_new, n_heads, use_rope)
    return kv_append_reference(qkv, k_cache, v_cache, cos, sin, pos, batch, n_new, n_heads)


def kv_append_reference(qkv, k_cache, v_cache, cos, sin, pos, batch, n_new, n_heads) -> Tensor:
    _, Hkv, Lmax, D = k_cache.shape
    H = n_heads
    p0 = int(pos.reshape(-1)[0])
    x = qkv.view(batch, n_new, H + 2 * Hkv, D)
    q, k, v = x[:, :, :H], x[:, :, H : H + Hkv], x[:, :, H + Hkv :]
    if cos is not None:
        tp = torch.arange(p0, p0 + n_new, device=qkv.device)
        q = F.apply_rope(q.float().transpose(1, 2), cos, sin, tp).transpose(1, 2).to(qkv.dtype)
        k = F.apply_rope(k.float().transpose(1, 2), cos, sin, tp).transpose(1, 2).to(qkv.dtype)
    n = max(0, min(n_new, Lmax - p0))
    k_cache[:, :, p0 : p0 + n] = k[:, :n].transpose(1, 2).to(k_cache.dtype)
    v_cache[:, :, p0 : p0 + n] = v[:, :n].transpose(1, 2).to(v_cache.dtype)
    return q.reshape(batch * n_new, H * D)


def decode_attention(q: Tensor, k_cache: Tensor, v_cache: Tensor, pos: Tensor, n_heads: int,
                     scale: float | None = None, n_new: int = 1) -> Tensor:
    """Attention of ``n_new`` new tokens per sequence (``q [B*n_new, H*D]``, already appended to the caches at
    positions ``pos .. pos + n_new - 1``) over the cache; token t sees keys ``0 .. pos + t``."""
    D = k_cache.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if q.is_cuda:
        return ops().decode_attn(q.contiguous(), k_cache, v_cache, pos, n_heads, scale, True, n_new)
    return decode_attention_reference(q, k_cache, v_cache, pos, n_heads, scale, n_new)


def decode_attention_reference(q, k_cache, v_cache, pos, n_heads, scale=None, n_new: int = 1) -> Tensor:
    B, Hkv, Lmax, D = k_cache.shape
    H, T = n_heads, n_new
    p0 = int(pos.reshape(-1)[0])
    L = min(p0 + T, Lmax)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    qf = q.float().view(B, T, Hkv, H // Hkv, D)
    k = k_cache[:, :, :L].float()
    v = v_cache[:, :, :L].float()
    s = torch.einsum("bthgd,bhld->bthgl", qf, k) * scale
    visible = torch.arange(L, device=q.device)[None, :] <= (p0 + torch.arange(T, device=q.device))[:, None]
    s = s.masked_fill(~visible[None, :, None, None, :], float("-inf"))
    o = torch.einsum("bthgl,bhld->bthgd", F.softmax(s, -1), v)
    return o.reshape(B * T, H * D).to(q.dtype)


def decode_attention_partials(q: Tensor, k_cache: Tensor, v_cache: Tensor, pos: Tensor, n_heads: int,
                              scale: float | None = None) -> Tensor:
    """Split-K decode attention without the combine: fp32 ``[B, H, nsplit, D + 2]`` = (o, m, l) per 256-key chunk
    (natural-log units; empty chunks have ``m = -inf``), consumed by :func:`decode_attn_proj`."""
    D = k_cache.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if q.is_cuda:
        return ops().decode_attn(q.contiguous(), k_cache, v_cache, pos, n_heads, scale, False)
    return decode_partials_reference(q, k_cache, v_cache, pos, n_heads, scale)


def decode_partials_reference(q, k_cache, v_cache, pos, n_heads, scale=None, chunk: int = 256) -> Tensor:
    B, Hkv, Lmax, D = k_cache.shape
    H = n_heads
    L = min(int(pos.reshape(-1)[0]) + 1, Lmax)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    ns = (Lmax + chunk - 1) // chunk
    out = torch.zeros(B, H, ns, D + 2, dtype=torch.float32, device=q.device)
    out[..., D] = -math.inf
    qf = q.float().view(B, Hkv, H // Hkv, D)
    for c in range(ns):
        s0, s1 = c * chunk, min(L, (c + 1) * chunk)
        if s0 >= s1:
            continue
        s = torch.einsum("bhgd,bhld->bhgl", qf, k_cache[:, :, s0:s1].float()) * scale
        m = s.amax(-1, keepdim=True)
        p = torch.exp(s - m)
        o = torch.einsum("bhgl,bhld->bhgd", p, v_cache[:, :, s0:s1].float())
        out[:, :, c, :D] = o.reshape(B, H, D)
        out[:, :, c, D] = m.reshape(B, H)
        out[:, :, c, D + 1] = p.sum(-1).reshape(B, H)
    return out


def decode_attn_proj(part: Tensor, w: Tensor) -> Tensor:
    """Output projection of the decode attention from its partials: ``combine(part) @ w.T`` (bf16 rounding of
    the combined rows as in the unfused path)."""
    if part.is_cuda:
        return ops().decode_attn_proj(part, w)
    B, H, _, D2 = part.shape
    D = D2 - 2
    m = part[..., D]
    mx = m.amax(-1, keepdim=True)
    c = torch.where(torch.isinf(m), torch.zeros_like(m), torch.exp(m - mx))
    o = (c[..., None] * part[..., :D]).sum(2) / (c * part[..., D + 1]).sum(-1, keepdim=True).clamp_min(1e-30)
    x = o.reshape(B, H * D).to(w.dtype)
    return (x.float() @ w.float().t()).to(w.dtype)


def decode_gemv(x: Tensor, w: Tensor, xd: Tensor | None = None, ln: Tensor | None = None, eps: float = 1e-5,
                swiglu: bool = False) -> tuple[Tensor, Tensor | None]:
    """Skinny projection of ``M <= 8`` decode rows (``csrc/decode_gemv.hip``): ``h = RMSNorm(x + xd) * ln``
    (each part optional), then ``y = h W^T`` or, with ``swiglu``, ``silu(h W1^T) * (h W3^T)`` for
    ``w = [W1; W3]``.  Returns ``(y, x + xd)`` (the second is ``None`` without ``xd``)."""
    if x.is_cuda:
        y, s = ops().decode_gemv(x, xd, ln, eps, w, 1 if swiglu else 0)
        return y, (s if xd is not None else None)
    return decode_gemv_reference(x, w, xd, ln, eps, swiglu)


def decode_gemv_reference(x, w, xd=None, ln=None, eps=1e-5, swiglu=False):
    """fp32 oracle with the kernel's rounding points (bf16 residual sum, bf16 GEMM outputs before SwiGLU)."""
    s = (x.float() + xd.float()).to(x.dtype) if xd is not None else x
    h = s.float()
    if ln is not None:
        h = (h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * ln.float()).to(x.dtype).float()
    y = (h @ w.float().t()).to(x.dtype)
    if swiglu:
        g, u = y.float().chunk(2, dim=-1)
        y = (g * torch.sigmoid(g) * u).to(x.dtype)
    return y, (s if xd is not None else None)


def decode_qkv(x: Tensor, w: Tensor, k_cache: Tensor, v_cache: Tensor, cos: Tensor | None, sin: Tensor | None,
               pos: Tensor, n_heads: int, xd: Tensor | None = None, ln: Tensor | None = None,
               eps: float = 1e-5) -> tuple[Tensor, Tensor | None]:
    """Fused decode QKV: ``qkv = RMSNorm(x + xd) W^T`` for one new token per sequence, RoPE at the device-side
    position, K / V written into the caches; returns ``(q [M, H*D], x + xd)``."""
    if x.is_cuda:
        use_rope = cos is not None
        c = cos if use_rope else x.new_empty(0, dtype=torch.float32)
        sn = sin if use_rope else x.new_empty(0, dtype=torch.float32)
        q, s = ops().decode_qkv(x, xd, ln, eps, w, k_cache, v_cache, c, sn, pos, n_heads, use_rope)
        return q, (s if xd is not None else None)
    qkv, s = decode_gemv_reference(x, w, xd, ln, eps)
    return kv_append_reference(qkv, k_cache, v_cache, cos, sin, pos, x.shape[0], 1, n_heads), s
