"""KV-cache serving kernels on the MI355X: ``kv_append`` / ``decode_attn`` (``ops/csrc/decode_attn.hip``) vs the
fp32 oracle, and the HIP-graph decode session vs the bf16 model's full forward."""

from __future__ import annotations

import copy
import math

import pytest
import torch

from bpe_transformer.models import DecodeSession, TransformerLM
from bpe_transformer.ops import decode as dec
from bpe_transformer.ops.reference import rope_tables

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("rope", [True, False])
def test_kv_append_matches_reference(gpu_device, D, rope):
    torch.manual_seed(0)
    B, T, H, Hkv, Lmax, p0 = 3, 5, 8, 2, 40, 7
    qkv = torch.randn(B * T, (H + 2 * Hkv) * D).bfloat16()
    cos, sin = rope_tables(D, Lmax, 10000.0) if rope else (None, None)
    pos = torch.tensor([p0], dtype=torch.int32)
    kc = torch.zeros(B, Hkv, Lmax, D, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    q_ref = dec.kv_append_reference(qkv.float(), kc, vc, cos, sin, pos, B, T, H)
    g = lambda t: None if t is None else t.to(gpu_device)  # noqa: E731
    kg, vg = torch.zeros_like(kc, device=gpu_device), torch.zeros_like(vc, device=gpu_device)
    q = dec.kv_append(qkv.to(gpu_device), kg, vg, g(cos), g(sin), pos.to(gpu_device), B, T, H)
    torch.cuda.synchronize()
    assert rel(q.cpu(), q_ref) < 1e-2
    assert rel(kg.cpu(), kc) < 1e-2
    assert torch.equal(vg.cpu(), vc)  # V is copied, not rotated
    assert kg[:, :, :p0].abs().sum() == 0 and kg[:, :, p0 + T :].abs().sum() == 0


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("G", [1, 2, 4, 8])
@pytest.mark.parametrize("L", [1, 200, 256, 257, 1000])
def test_decode_attention_matches_reference(gpu_device, D, G, L):
    torch.manual_seed(L + G)
    B, Hkv, Lmax = 2, 2, 1024
    H = Hkv * G
    q = torch.randn(B, H * D).bfloat16()
    kc = torch.randn(B, Hkv, Lmax, D).bfloat16()
    vc = torch.randn(B, Hkv, Lmax, D).bfloat16()
    pos = torch.tensor([L - 1], dtype=torch.int32)
    ref = dec.decode_attention_reference(q.float(), kc, vc, pos, H, 1.0 / math.sqrt(D))
    out = dec.decode_attention(q.to(gpu_device), kc.to(gpu_device), vc.to(gpu_device), pos.to(gpu_device), H)
    assert rel(out.cpu(), ref) < 2e-2, rel(out.cpu(), ref)


def test_decode_attention_large_scores(gpu_device):
    """One dominant key per chunk boundary: the cross-chunk combine must rescale correctly."""
    torch.manual_seed(5)
    B, H, Hkv, D, Lmax = 1, 4, 4, 64, 768
    q = torch.randn(B, H * D).bfloat16()
    kc = torch.randn(B, Hkv, Lmax, D).bfloat16() * 0.1
    vc = torch.randn(B, Hkv, Lmax, D).bfloat16()
    kc[:, :, 600] = q.view(B, H, D) * 4  # a key in the third chunk dominates
    pos = torch.tensor([Lmax - 1], dtype=torch.int32)
    ref = dec.decode_attention_reference(q.float(), kc, vc, pos, H)
    out = dec.decode_attention(q.to(gpu_device), kc.to(gpu_device), vc.to(gpu_device), pos.to(gpu_device), H)
    assert rel(out.cpu(), ref) < 2e-2


def _bf16_model(gpu_device, **kw):
    torch.manual_seed(0)
    cfg = dict(vocab_size=1000, context_length=256, d_model=256, num_layers=2, num_heads=4, d_ff=512)
    cfg.update(kw)
    return TransformerLM(**cfg).to(gpu_device, torch.bfloat16).eval()


@pytest.mark.parametrize("kw", [{}, {"num_kv_heads": 2}, {"remove_rope": True}])
@pytest.mark.parametrize("use_graph", [True, False])
def test_session_matches_full_forward(gpu_device, kw, use_graph):
    model = _bf16_model(gpu_device, **kw)
    ids = torch.randint(0, 1000, (3, 40), device=gpu_device)
    sess = DecodeSession(model, 3, max_len=64, use_graph=use_graph)
    assert sess.fast
    with torch.no_grad():
        full = model(ids).float()
        got = [sess.prefill(ids[:, :30])]
        for t in range(30, 40):
            got.append(sess.decode(ids[:, t]))
    torch.cuda.synchronize()
    want = [full[:, 29]] + [full[:, t] for t in range(30, 40)]
    for i, (a, b) in enumerate(zip(got, want)):
        assert rel(a, b) < 3e-2, (i, rel(a, b))


def test_graph_replay_equals_eager(gpu_device):
    model = _bf16_model(gpu_device)
    ids = torch.randint(0, 1000, (2, 24), device=gpu_device)
    a = DecodeSession(model, 2, max_len=32, use_graph=True)
    b = DecodeSession(model, 2, max_len=32, use_graph=False)
    with torch.no_grad():
        a.prefill(ids[:, :16])
        b.prefill(ids[:, :16])
        for t in range(16, 24):
            la, lb = a.decode(ids[:, t]), b.decode(ids[:, t])
            assert rel(la, lb) < 1e-3
    assert torch.equal(a.cache.k, b.cache.k) and torch.equal(a.cache.v, b.cache.v)


def test_generate_uses_cache_on_gpu(gpu_device):
    model = _bf16_model(gpu_device)
    prompt = torch.randint(0, 1000, (2, 8), device=gpu_device)
    out = model.generate(prompt, 12, temperature=0.0)
    assert out.shape == (2, 20) and torch.equal(out[:, :8], prompt)
    ref = copy.deepcopy(model)
    first = ref.generate(prompt, 1, temperature=0.0, use_cache=False)
    assert torch.equal(out[:, 8], first[:, 8])


@pytest.mark.parametrize("M", [1, 3, 8, 13, 16])
@pytest.mark.parametrize("K,N", [(256, 1000), (768, 2304), (2048, 512)])
@pytest.mark.parametrize("prologue", [False, True])
@pytest.mark.parametrize("swiglu", [False, True])
def test_decode_gemv_matches_reference(gpu_device, M, K, N, prologue, swiglu):
    torch.manual_seed(M * 7 + K)
    x = torch.randn(M, K).bfloat16()
    w = (torch.randn(N, K) / math.sqrt(K)).bfloat16()
    xd = torch.randn(M, K).bfloat16() if prologue else None
    ln = (1 + 0.1 * torch.randn(K)).bfloat16() if prologue else None
    y_ref, s_ref = dec.decode_gemv_reference(x, w, xd, ln, 1e-5, swiglu)
    g = lambda t: None if t is None else t.to(gpu_device)  # noqa: E731
    y, s = dec.decode_gemv(g(x), g(w), g(xd), g(ln), 1e-5, swiglu)
    torch.cuda.synchronize()
    assert y.shape == y_ref.shape
    assert rel(y.cpu(), y_ref) < 2e-2, rel(y.cpu(), y_ref)
    if prologue:
        assert torch.equal(s.cpu(), s_ref)


@pytest.mark.parametrize("D,G", [(64, 1), (64, 4), (128, 2)])
@pytest.mark.parametrize("rope", [True, False])
def test_decode_qkv_matches_reference(gpu_device, D, G, rope):
    torch.manual_seed(D + G)
    M, Hkv, Lmax, p0, K = 4, 2, 48, 17, 512
    H = Hkv * G
    x = torch.randn(M, K).bfloat16()
    xd = torch.randn(M, K).bfloat16()
    ln = (1 + 0.1 * torch.randn(K)).bfloat16()
    w = (torch.randn((H + 2 * Hkv) * D, K) / math.sqrt(K)).bfloat16()
    cos, sin = rope_tables(D, Lmax, 10000.0) if rope else (None, None)
    pos = torch.tensor([p0], dtype=torch.int32)
    kc = torch.zeros(M, Hkv, Lmax, D, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    q_ref, s_ref = dec.decode_qkv(x, w, kc, vc, cos, sin, pos, H, xd, ln)
    g = lambda t: None if t is None else t.to(gpu_device)  # noqa: E731
    kg, vg = torch.zeros_like(kc, device=gpu_device), torch.zeros_like(vc, device=gpu_device)
    q, s = dec.decode_qkv(g(x), g(w), kg, vg, g(cos), g(sin), g(pos), H, g(xd), g(ln))
    torch.cuda.synchronize()
    assert rel(q.cpu(), q_ref) < 2e-2
    assert rel(kg.cpu(), kc) < 2e-2 and rel(vg.cpu(), vc) < 2e-2
    assert torch.equal(s.cpu(), s_ref)
    assert kg[:, :, :p0].abs().sum() == 0 and kg[:, :, p0 + 1 :].abs().sum() == 0


def test_gemv_decode_matches_library_decode(gpu_device, monkeypatch):
    """The fused skinny-GEMM decode step (batch <= 8) agrees with the hipBLASLt + elementwise-kernel step."""
    from bpe_transformer.models import generation

    model = _bf16_model(gpu_device, num_kv_heads=2)
    ids = torch.randint(0, 1000, (12, 24), device=gpu_device)
    outs = []
    for cap in (16, 0):
        monkeypatch.setattr(generation, "_GEMV_MAX_BATCH", cap)
        sess = DecodeSession(model, 12, max_len=32, use_graph=True)
        with torch.no_grad():
            sess.prefill(ids[:, :16])
            outs.append([sess.decode(ids[:, t]) for t in range(16, 24)])
    for a, b in zip(*outs):
        assert rel(a, b) < 2e-2, rel(a, b)


@pytest.mark.parametrize("D,G", [(64, 1), (64, 4), (128, 2)])
@pytest.mark.parametrize("L", [1, 300, 777])
@pytest.mark.parametrize("B", [1, 5])
def test_decode_attn_proj_matches_reference(gpu_device, D, G, L, B):
    """Split-K partials -> output projection with the combine in its prologue vs the fp32 oracle."""
    torch.manual_seed(L + G + B)
    Hkv, Lmax, N = 2, 1024, 384
    H = Hkv * G
    q = torch.randn(B, H * D).bfloat16()
    kc = torch.randn(B, Hkv, Lmax, D).bfloat16()
    vc = torch.randn(B, Hkv, Lmax, D).bfloat16()
    w = (torch.randn(N, H * D) / math.sqrt(H * D)).bfloat16()
    pos = torch.tensor([L - 1], dtype=torch.int32)
    o_ref = dec.decode_attention_reference(q.float(), kc, vc, pos, H).bfloat16()
    y_ref = o_ref.float() @ w.float().t()
    g = lambda t: t.to(gpu_device)  # noqa: E731
    part = dec.decode_attention_partials(g(q), g(kc), g(vc), g(pos), H)
    y = dec.decode_attn_proj(part, g(w))
    torch.cuda.synchronize()
    assert part.shape == (B, H, Lmax // 256, D + 2)
    assert rel(y.cpu(), y_ref) < 2e-2, rel(y.cpu(), y_ref)


@pytest.mark.parametrize("D,G,T", [(64, 1, 2), (64, 1, 5), (64, 2, 4), (128, 4, 2), (64, 1, 8)])
@pytest.mark.parametrize("p0", [0, 250, 700])
def test_multi_token_decode_attention(gpu_device, D, G, T, p0):
    """T new tokens per sequence in one decode_attn (chunked prefill into a filled cache): per-token causal."""
    torch.manual_seed(p0 + T)
    B, Hkv, Lmax = 2, 2, 1024
    H = Hkv * G
    q = torch.randn(B * T, H * D).bfloat16()
    kc = torch.randn(B, Hkv, Lmax, D).bfloat16()
    vc = torch.randn(B, Hkv, Lmax, D).bfloat16()
    pos = torch.tensor([p0], dtype=torch.int32)
    ref = dec.decode_attention_reference(q.float(), kc, vc, pos, H, None, T)
    g = lambda t: t.to(gpu_device)  # noqa: E731
    out = dec.decode_attention(g(q), g(kc), g(vc), g(pos), H, n_new=T)
    torch.cuda.synchronize()
    assert rel(out.cpu(), ref) < 2e-2, rel(out.cpu(), ref)


@pytest.mark.parametrize("kw", [{}, {"num_kv_heads": 2}])
def test_append_to_filled_cache_matches_full_forward(gpu_device, kw):
    """prefill, then a 7-token chunk appended to the filled cache (multi-token decode steps), then decode."""
    model = _bf16_model(gpu_device, **kw)
    ids = torch.randint(0, 1000, (3, 34), device=gpu_device)
    sess = DecodeSession(model, 3, max_len=64)
    with torch.no_grad():
        full = model(ids).float()
        sess.prefill(ids[:, :20])
        got = [sess.prefill(ids[:, 20:27])]
        for t in range(27, 34):
            got.append(sess.decode(ids[:, t]))
    torch.cuda.synchronize()
    want = [full[:, 26]] + [full[:, t] for t in range(27, 34)]
    for i, (a, b) in enumerate(zip(got, want)):
        assert rel(a, b) < 3e-2, (i, rel(a, b))
