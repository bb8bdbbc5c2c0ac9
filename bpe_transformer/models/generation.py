"""KV-cache inference: prefill + single-token decode, HIP-graph-captured on MI355X.

The reference has no inference engine (SURVEY §1 lists serving among the
absent layers; its only "generation" is the contract model's logits,
``tests/adapters.py:282-361``).  :meth:`TransformerLM.generate` used to re-run
the whole prefix for each new token; :class:`DecodeSession` keeps a KV cache
instead:

* **prefill** (``T`` prompt tokens, empty cache): the training kernels --
  RMSNorm, the fused [Wq;Wk;Wv] GEMM, flash attention with fused RoPE -- plus
  ``kv_append``, which writes the roped K and the V of all ``T`` tokens into
  the cache in one launch;
* **append** to a filled cache (a new turn of a conversation, draft tokens to
  verify): steps of up to ``8 / G`` tokens per sequence, each a multi-token
  ``kv_append`` + ``decode_attn`` in which token ``t`` sees the cache and its
  own causal prefix (``pos + t``), instead of one decode step per token;
* **decode** (one token per sequence): ``kv_append`` (RoPE at the device-side
  position, cache write, roped q) -> ``decode_attn`` (split-K flash-decoding
  over the cache) for every layer, residual adds fused into the next RMSNorm,
  then the LM head.  The position lives in a device int32 tensor, so the whole
  step has static shapes and is captured once into a HIP graph
  (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replayed per token: one
  graph launch instead of ~10 kernel launches per layer.

Cache layout: ``k, v: [num_layers, B, Hkv, Lmax, D]`` bf16 (RoPE already
applied to K), i.e. each (sequence, kv head) is one contiguous ``Lmax x D``
slab the decode kernel streams.  GPT-2-small at Lmax 1024 needs 36 MiB per
sequence, so a 288 GB MI355X holds thousands of sequences.

On the CPU, in fp32, or with the reference ablations (post-norm, no RMSNorm,
non-SwiGLU FFN) the same session runs the oracle math over the same cache.
"""

from __future__ import annotations

import math
import os

import torch
from torch import Tensor

from ..ops import reference as F

# decode steps of up to this many sequences run on the fused skinny-GEMM kernels (they take up to 16 -- one MFMA
# column block -- but every workgroup re-normalises all rows in its prologue, so past ~12 rows the library
# GEMMs (hipBLASLt) win: GPT-2-small at 16 sequences 0.737 vs 0.699 ms, at 8 0.499 vs 0.672)
_GEMV_MAX_BATCH = int(os.environ.get("BPE_DECODE_GEMV_MAX_BATCH", "8"))


def _gemv_ok(m: int, k: int) -> bool:
    """Mirror of ``gemv_ok`` (csrc/decode_gemv.hip): rows x K that the skinny kernels take."""
    if m < 1 or k % 8:
        return False
    mfma = m <= 16 and k % 32 == 0 and m * (k + 8) * 2 + 4352 <= 160 * 1024
    if m > 8:
        return mfma
    rows = 1 << (m - 1).bit_length()  # the VALU kernel's LDS holds m rounded up to 1, 2, 4 or 8 rows
    return rows * k * 2 <= 160 * 1024 or mfma


class KVCache:
    """Per-layer K/V caches ``[L, B, Hkv, Lmax, D]`` plus the device-side fill position."""

    def __init__(self, num_layers: int, batch: int, num_kv_heads: int, max_len: int, head_dim: int, device=None,
                 dtype=torch.bfloat16):
        shape = (num_layers, batch, num_kv_heads, max_len, head_dim)
        self.k = torch.zeros(shape, device=device, dtype=dtype)
        self.v = torch.zeros(shape, device=device, dtype=dtype)
        self.pos = torch.zeros(1, device=device, dtype=torch.int32)  # tokens already cached
        self.length = 0  # host mirror of pos (the host never reads pos back)
        self.max_len = max_len
        self.batch = batch

    def reset(self) -> None:
        self.pos.zero_()
        self.length = 0

    def nbytes(self) -> int:
        return 2 * self.k.numel() * self.k.element_size()


def _sample(logits: Tensor, temperature: float, top_p: float | None, generator) -> Tensor:
    """Next token per row of ``logits [B, V]`` (greedy when ``temperature <= 0``); returns ``[B]`` int64."""
    logits = logits.float()
    if temperature <= 0:
        return logits.argmax(-1)
    probs = torch.softmax(logits / temperature, dim=-1)
    if top_p is not None and top_p < 1.0:
        sp, si = probs.sort(dim=-1, descending=True)
        keep = sp.cumsum(-1) - sp < top_p
        sp = sp * keep
        probs = torch.zeros_like(probs).scatter_(-1, si, sp)
        probs = probs / probs.sum(-1, keepdim=True)
    return torch.multinomial(probs, 1, generator=generator).squeeze(-1)


class DecodeSession:
    """Incremental decoding of ``batch`` sequences with a KV cache.

    ``prefill(ids [B, T])`` and ``decode(ids [B])`` return the next-token logits ``[B, V]`` of the last position.
    With ``use_graph`` (GPU only) the decode step is captured into a HIP graph on first use and replayed after.
    """

    def __init__(self, model, batch: int, max_len: int | None = None, use_graph: bool = True):
        self.model = model
        cfg = model.config
        self.batch = batch
        self.max_len = max_len or model.context_length
        blk = model.layers[0] if len(model.layers) else None
        attn = blk.attn if blk is not None else None
        self.H = attn.num_heads if attn else cfg.num_heads
        self.Hkv = attn.num_kv_heads if attn else cfg.num_heads
        self.D = attn.d_k if attn else cfg.d_model // cfg.num_heads
        if attn is not None and attn.rope is not None:
            assert self.max_len <= attn.rope.max_seq_len, "KV cache longer than the RoPE table (context_length)"
        p = model.lm_head.weight
        self.device = p.device
        self.cache = KVCache(len(model.layers), batch, self.Hkv, self.max_len, self.D, self.device, p.dtype)
        self.fast = self._fast_ok()
        self.use_graph = use_graph and self.fast
        self._graph = None
        if self.fast:
            self._prepare_weights()

    # ------------------------------------------------------------------ setup
    def _fast_ok(self) -> bool:
        m = self.model
        if not (self.device.type == "cuda" and m.lm_head.weight.dtype == torch.bfloat16 and len(m.layers)):
            return False
        from .. import ops

        for layer in m.layers:
            if layer.use_post_norm or layer.remove_rmsnorm or layer.ffn_type != "swiglu":
                return False
        G = self.H // self.Hkv
        return self.D in ops.attention.SUPPORTED_HEAD_DIMS and G in (1, 2, 4, 8) and self.H % self.Hkv == 0

    def _prepare_weights(self) -> None:
        from .fused_block import _cat_weights

        self._w = []
        for layer in self.model.layers:
            a, f = layer.attn, layer.ffn
            self._w.append((
                layer.ln1.weight.detach(), _cat_weights([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight]),
                a.output_proj.weight.detach(), layer.ln2.weight.detach(), _cat_weights([f.w1.weight, f.w3.weight]),
                f.w2.weight.detach(), layer.ln1.eps,
            ))
        rope = self.model.layers[0].attn.rope
        if rope is not None:
            self._cos, self._sin = rope.cos.float().contiguous(), rope.sin.float().contiguous()
        else:
            self._cos = self._sin = None

    def reset(self) -> None:
        self.cache.reset()

    @property
    def length(self) -> int:
        return self.cache.length

    # ------------------------------------------------------------------ public API
    @torch.no_grad()
    def prefill(self, ids: Tensor) -> Tensor:
        """Append ``ids [B, T]`` to the cache; returns the logits ``[B, V]`` after the last token."""
        ids = ids.to(self.device)
        B, T = ids.shape
        assert B == self.batch, f"session batch is {self.batch}, got {B}"
        assert self.cache.length + T <= self.max_len, "KV cache full"
        if self.fast and self.cache.length == 0 and T > 1:
            out = self._forward_fast(ids, prefill=True)
        elif self.fast:
            # appending to a filled cache (multi-turn serving, speculative verification): chunks of up to
            # 8 / G tokens per step, each attending the cache plus its own causal prefix in one decode_attn
            out = None
            step = max(1, 8 // (self.H // self.Hkv))
            for t in range(0, T, step):
                out = self._forward_fast(ids[:, t : t + step], prefill=False)
        else:
            out = self._forward_reference(ids)
        self.cache.length += T
        return out

    @torch.no_grad()
    def decode(self, ids: Tensor) -> Tensor:
        """Append one token per sequence (``ids [B]``); returns the next logits ``[B, V]``."""
        assert self.cache.length + 1 <= self.max_len, "KV cache full"
        ids = ids.reshape(self.batch, 1).to(self.device)
        if not self.use_graph:
            out = self._forward_fast(ids, prefill=False) if self.fast else self._forward_reference(ids)
        else:
            if self._graph is None:
                self._capture()
            self._static_ids.copy_(ids)
            self._graph.replay()
            out = self._static_logits.clone()  # the graph's output buffer is rewritten by the next replay
        self.cache.length += 1
        return out

    @torch.no_grad()
    def generate(self, prompt: Tensor, max_new_tokens: int, temperature: float = 1.0, top_p: float | None = None,
                 eos_token_id: int | None = None, generator: torch.Generator | None = None) -> Tensor:
        """``prompt [B, S]`` -> ``[B, S + n]`` (stops early once every row emitted ``eos_token_id``)."""
        self.reset()
        logits = self.prefill(prompt)
        outs = [prompt.to(self.device)]
        done = None
        for i in range(max_new_tokens):
            nxt = _sample(logits, temperature, top_p, generator)
            outs.append(nxt[:, None])
            if eos_token_id is not None:
                hit = nxt == eos_token_id
                done = hit if done is None else (done | hit)
                if bool(done.all()):
                    break
            if i + 1 < max_new_tokens:
                logits = self.decode(nxt)
        return torch.cat(outs, 1)

    # ------------------------------------------------------------------ HIP path
    def _capture(self) -> None:
        """Capture one decode step (all layers + LM head) into a HIP graph.  The warm-up run writes the cache at
        the current position (rewritten by the first replay) and the position is restored afterwards."""
        self._static_ids = torch.zeros(self.batch, 1, dtype=torch.long, device=self.device)
        pos0 = self.cache.pos.clone()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._forward_fast(self._static_ids, prefill=False)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.cache.pos.copy_(pos0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._static_logits = self._forward_fast(self._static_ids, prefill=False)
        self.cache.pos.copy_(pos0)  # capture does not execute, but keep the invariant explicit
        self._graph = g

    def _forward_fast(self, ids: Tensor, prefill: bool) -> Tensor:
        if not prefill and ids.shape[1] == 1 and ids.shape[0] <= _GEMV_MAX_BATCH and self._gemv_fits(ids.shape[0]):
            return self._decode_gemv(ids)
        from ..ops._ext import ops as hip

        h = hip()
        m = self.model
        B, T = ids.shape
        H, Hkv, D = self.H, self.Hkv, self.D
        scale = 1.0 / math.sqrt(D)
        kc, vc, pos = self.cache.k, self.cache.v, self.cache.pos
        use_rope = self._cos is not None
        cos = self._cos if use_rope else kc.new_empty(0, dtype=torch.float32)
        sin = self._sin if use_rope else kc.new_empty(0, dtype=torch.float32)
        xr = m.token_embeddings(ids).reshape(B * T, -1)
        xd = None
        for li, (ln1, wqkv, wo, ln2, w13, w2, eps) in enumerate(self._w):
            if xd is None:
                h1, _ = h.rmsnorm_fwd(xr, ln1, eps)
            else:
                xr, h1, _ = h.add_rmsnorm_fwd(xr, xd, ln1, eps)
            qkv = torch.matmul(h1, wqkv.t())
            if prefill:
                q, k, v = qkv[:, : H * D], qkv[:, H * D : (H + Hkv) * D], qkv[:, (H + Hkv) * D :]
                o, _ = h.fa_fwd(q, k, v, cos, sin, B, T, H, Hkv, D, True, use_rope, scale)
                h.kv_append(qkv, kc[li], vc[li], cos, sin, pos, B, T, H, use_rope)
            else:
                q = h.kv_append(qkv, kc[li], vc[li], cos, sin, pos, B, T, H, use_rope)
                o = h.decode_attn(q, kc[li], vc[li], pos, H, scale, True, T)
            g1 = torch.matmul(o, wo.t())
            xr, h2, _ = h.add_rmsnorm_fwd(xr, g1, ln2, eps)
            a = h.swiglu_fwd(torch.matmul(h2, w13.t()))
            xd = torch.matmul(a, w2.t())
        if T > 1:  # only the last position's logits are needed
            xr = xr.view(B, T, -1)[:, -1].contiguous()
            xd = xd.view(B, T, -1)[:, -1].contiguous()
        fin = m.ln_final
        _, hf, _ = h.add_rmsnorm_fwd(xr, xd, fin.weight, fin.eps)
        logits = torch.matmul(hf, m.lm_head.weight.t())
        pos.add_(T)
        return logits

    def _gemv_fits(self, m: int) -> bool:
        cfg = self.model.config
        return all(_gemv_ok(m, k) for k in (cfg.d_model, self.H * self.D, self._w[0][5].shape[1]))

    def _decode_gemv(self, ids: Tensor) -> Tensor:
        """Decode step for batch <= 16 on the fused skinny-GEMM kernels (``csrc/decode_gemv.hip``): per layer
        qkv (+RMSNorm, +RoPE, +cache write) -> split-K decode attention -> Wo (+ the split combine) -> [W1; W3]
        (+residual add, +RMSNorm, +SwiGLU) -> W2; the residual add of W2's output is folded into the next layer's
        QKV prologue: 5 launches per layer."""
        from ..ops._ext import ops as hip

        h = hip()
        m = self.model
        H = self.H
        scale = 1.0 / math.sqrt(self.D)
        kc, vc, pos = self.cache.k, self.cache.v, self.cache.pos
        use_rope = self._cos is not None
        cos = self._cos if use_rope else kc.new_empty(0, dtype=torch.float32)
        sin = self._sin if use_rope else kc.new_empty(0, dtype=torch.float32)
        xr = m.token_embeddings(ids).reshape(ids.shape[0], -1)
        xd = None
        for li, (ln1, wqkv, wo, ln2, w13, w2, eps) in enumerate(self._w):
            q, s = h.decode_qkv(xr, xd, ln1, eps, wqkv, kc[li], vc[li], cos, sin, pos, H, use_rope)
            if xd is not None:
                xr = s
            part = h.decode_attn(q, kc[li], vc[li], pos, H, scale, False)
            g1 = h.decode_attn_proj(part, wo)  # the flash-decoding combine runs in Wo's prologue
            a, xr = h.decode_gemv(xr, g1, ln2, eps, w13, 1)
            xd, _ = h.decode_gemv(a, None, None, 0.0, w2, 0)
        fin = m.ln_final
        logits, _ = h.decode_gemv(xr, xd, fin.weight, fin.eps, m.lm_head.weight, 0)
        pos.add_(1)
        return logits

    # ------------------------------------------------------------------ oracle path
    def _forward_reference(self, ids: Tensor) -> Tensor:
        """Plain-PyTorch math over the same cache (any dtype / device / ablation)."""
        m = self.model
        B, T = ids.shape
        p0 = self.cache.length
        H, Hkv, D = self.H, self.Hkv, self.D
        x = m.token_embeddings(ids)
        tp = torch.arange(p0, p0 + T, device=ids.device)
        mask = F.causal_mask(T, p0 + T, device=ids.device)
        for li, layer in enumerate(m.layers):
            attn = layer.attn

            def attend(z: Tensor) -> Tensor:
                q = attn.q_proj(z).view(B, T, H, D).transpose(1, 2)
                k = attn.k_proj(z).view(B, T, Hkv, D).transpose(1, 2)
                v = attn.v_proj(z).view(B, T, Hkv, D).transpose(1, 2)
                if attn.rope is not None:
                    q = attn.rope(q, tp)
                    k = attn.rope(k, tp)
                self.cache.k[li, :, :, p0 : p0 + T] = k.to(self.cache.k.dtype)
                self.cache.v[li, :, :, p0 : p0 + T] = v.to(self.cache.v.dtype)
                kk = self.cache.k[li, :, :, : p0 + T].to(q.dtype)
                vv = self.cache.v[li, :, :, : p0 + T].to(q.dtype)
                if Hkv != H:
                    kk = kk.repeat_interleave(H // Hkv, dim=1)
                    vv = vv.repeat_interleave(H // Hkv, dim=1)
                o = F.scaled_dot_product_attention(q, kk, vv, mask)
                return attn.output_proj(o.transpose(1, 2).reshape(B, T, H * D))

            if layer.use_post_norm:
                x = layer.ln1(x + attend(x))
                x = layer.ln2(x + layer.ffn(x))
            else:
                x = x + attend(layer.ln1(x))
                x = x + layer.ffn(layer.ln2(x))
        logits = m.lm_head(m.ln_final(x[:, -1]))
        self.cache.pos.add_(T)
        return logits
