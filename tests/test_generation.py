"""KV-cache inference (``models/generation.py``, ``ops/decode.py``) on the CPU oracle path.

The reference has no inference engine; the parity target is the contract model itself
(``tests/adapters.py:282-361``): decoding token by token through the cache must give the logits of running the
full prefix through ``TransformerLM.forward``.
"""

from __future__ import annotations

import math

import pytest
import torch

from bpe_transformer.models import DecodeSession, TransformerLM
from bpe_transformer.ops import decode as dec
from bpe_transformer.ops.attention import attention_qkv_reference
from bpe_transformer.ops.reference import rope_tables

VARIANTS = {
    "default": {},
    "gqa": {"num_kv_heads": 2},
    "no_rope": {"remove_rope": True},
    "post_norm": {"use_post_norm": True},
    "no_rmsnorm": {"remove_rmsnorm": True},
    "gelu_ffn": {"ffn_type": "gelu"},
}


def _model(**kw):
    torch.manual_seed(0)
    cfg = dict(vocab_size=97, context_length=32, d_model=64, num_layers=2, num_heads=4, d_ff=96)
    cfg.update(kw)
    return TransformerLM(**cfg).eval()


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_cached_decode_matches_full_forward(variant):
    model = _model(**VARIANTS[variant])
    ids = torch.randint(0, 97, (3, 20))
    sess = DecodeSession(model, 3)
    with torch.no_grad():
        full = model(ids)
        got = [sess.prefill(ids[:, :6])]
        for t in range(6, 20):
            got.append(sess.decode(ids[:, t]))
    assert sess.length == 20
    want = torch.stack([full[:, 5]] + [full[:, t] for t in range(6, 20)])
    assert torch.allclose(torch.stack(got), want, atol=1e-4, rtol=1e-4)


def test_chunked_prefill_matches_single_prefill():
    model = _model(num_kv_heads=2)
    ids = torch.randint(0, 97, (2, 12))
    a, b = DecodeSession(model, 2), DecodeSession(model, 2)
    with torch.no_grad():
        la = a.prefill(ids)
        b.prefill(ids[:, :5])
        lb = b.prefill(ids[:, 5:])
    assert torch.allclose(la, lb, atol=1e-5)
    assert torch.equal(a.cache.k, b.cache.k) or torch.allclose(a.cache.k, b.cache.k, atol=1e-6)


def test_generate_with_cache_equals_recompute():
    model = _model()
    prompt = torch.randint(0, 97, (2, 5))
    a = model.generate(prompt, 10, temperature=0.0, use_cache=True)
    b = model.generate(prompt, 10, temperature=0.0, use_cache=False)
    assert a.shape == (2, 15) and torch.equal(a, b)
    one = model.generate(prompt[0], 4, temperature=0.0)
    assert one.shape == (9,) and torch.equal(one, a[0, :9])


def test_generate_sampling_reproducible():
    model = _model()
    prompt = torch.randint(0, 97, (2, 4))
    outs = []
    for _ in range(2):
        g = torch.Generator().manual_seed(7)
        outs.append(model.generate(prompt, 8, temperature=0.8, top_p=0.9, generator=g))
    assert torch.equal(outs[0], outs[1])


def test_generate_eos_stops():
    model = _model()
    prompt = torch.randint(0, 97, (1, 4))
    first = model.generate(prompt, 1, temperature=0.0)[0, -1].item()
    out = model.generate(prompt, 10, temperature=0.0, eos_token_id=first)
    assert out.shape == (1, 5)


@pytest.mark.parametrize("rope", [True, False])
def test_kv_append_and_decode_reference_match_attention(rope):
    """Oracle ops: appending a whole sequence, then attending from the last position == causal attention."""
    torch.manual_seed(1)
    B, S, H, Hkv, D = 2, 9, 4, 2, 16
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D)
    cos, sin = rope_tables(D, 16, 10000.0) if rope else (None, None)
    kc = torch.zeros(B, Hkv, 16, D)
    vc = torch.zeros_like(kc)
    pos = torch.zeros(1, dtype=torch.int32)
    q = dec.kv_append(qkv, kc, vc, cos, sin, pos, B, S, H)
    assert q.shape == (B * S, H * D)
    want = attention_qkv_reference(qkv, B, S, H, Hkv, D, cos, sin, True).view(B, S, H * D)
    pos.fill_(S - 1)
    o = dec.decode_attention(q.view(B, S, H * D)[:, -1].contiguous(), kc, vc, pos, H, 1.0 / math.sqrt(D))
    assert torch.allclose(o, want[:, -1], atol=1e-5)


def test_decode_qkv_oracle_matches_kv_append():
    """CPU oracle of the fused decode QKV equals RMSNorm -> projection -> kv_append."""
    torch.manual_seed(0)
    M, K, H, Hkv, D, Lmax = 2, 64, 4, 2, 16, 12
    x, xd = torch.randn(M, K), torch.randn(M, K)
    ln = 1 + 0.1 * torch.randn(K)
    w = torch.randn((H + 2 * Hkv) * D, K)
    cos, sin = rope_tables(D, Lmax, 10000.0)
    pos = torch.tensor([5], dtype=torch.int32)
    kc, vc = torch.zeros(M, Hkv, Lmax, D), torch.zeros(M, Hkv, Lmax, D)
    q, s = dec.decode_qkv(x, w, kc, vc, cos, sin, pos, H, xd, ln)
    assert torch.allclose(s, x + xd)
    hn = s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + 1e-5) * ln
    k2, v2 = torch.zeros_like(kc), torch.zeros_like(vc)
    q2 = dec.kv_append_reference(hn @ w.t(), k2, v2, cos, sin, pos, M, 1, H)
    assert torch.allclose(q, q2, atol=1e-5) and torch.allclose(kc, k2, atol=1e-5) and torch.equal(vc, v2)
    y, _ = dec.decode_gemv(x, torch.randn(2 * 8, K), swiglu=True)
    assert y.shape == (M, 8)


def test_decode_partials_combine_to_attention():
    """CPU oracle: merging the split-K partials (decode_attn_proj with an identity weight) equals attention."""
    torch.manual_seed(1)
    B, H, Hkv, D, Lmax = 2, 4, 2, 16, 600
    q = torch.randn(B, H * D)
    kc, vc = torch.randn(B, Hkv, Lmax, D), torch.randn(B, Hkv, Lmax, D)
    pos = torch.tensor([530], dtype=torch.int32)
    part = dec.decode_attention_partials(q, kc, vc, pos, H)
    assert part.shape == (B, H, 3, D + 2)
    eye = torch.eye(H * D)
    got = dec.decode_attn_proj(part, eye)
    want = dec.decode_attention_reference(q, kc, vc, pos, H)
    assert torch.allclose(got, want, atol=1e-5)


def test_multi_token_decode_attention_oracle_is_per_token_causal():
    """n_new tokens in one call == n_new single-token calls with the position advanced each time."""
    torch.manual_seed(2)
    B, H, Hkv, D, Lmax, T, p0 = 2, 4, 2, 16, 40, 3, 17
    q = torch.randn(B * T, H * D)
    kc, vc = torch.randn(B, Hkv, Lmax, D), torch.randn(B, Hkv, Lmax, D)
    got = dec.decode_attention(q, kc, vc, torch.tensor([p0], dtype=torch.int32), H, n_new=T).view(B, T, H * D)
    for t in range(T):
        want = dec.decode_attention(q.view(B, T, -1)[:, t], kc, vc, torch.tensor([p0 + t], dtype=torch.int32), H)
        assert torch.allclose(got[:, t], want, atol=1e-5)
