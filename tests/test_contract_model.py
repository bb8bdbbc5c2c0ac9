"""Model contract tests (reference contracts K1-K12).

Two kinds:
  * snapshot tests against the reference's ``tests/_snapshots/*.npz`` for
    everything that needs no weights (SDPA 3-D/4-D, RoPE, SiLU); the
    weight-dependent snapshots need the reference's ``model.pt`` blob, which
    is missing from the mirror -- those run when it is present, else skip;
  * oracle tests: every module against an independent einsum/loop formula of
    its contract, with random weights in the reference's state-dict format.
"""

from __future__ import annotations

import math

import pytest
import torch

from .adapters import (
    run_embedding,
    run_linear,
    run_multihead_self_attention,
    run_multihead_self_attention_with_rope,
    run_rmsnorm,
    run_rope,
    run_scaled_dot_product_attention,
    run_silu,
    run_swiglu,
    run_transformer_block,
    run_transformer_lm,
)


# ---------------------------------------------------------------- snapshots (no weights needed)
def test_scaled_dot_product_attention(numpy_snapshot, q, k, v, mask):
    numpy_snapshot.assert_match(run_scaled_dot_product_attention(q, k, v, mask), atol=1e-6)


def test_4d_scaled_dot_product_attention(numpy_snapshot, q, k, v, mask):
    q4, k4, v4 = (x.reshape(2, 2, *x.shape[1:]) for x in (q, k, v))
    m4 = mask.reshape(2, 2, *mask.shape[1:])
    numpy_snapshot.assert_match(run_scaled_dot_product_attention(q4, k4, v4, m4), atol=1e-6)


@pytest.mark.parametrize("mdtype", [torch.int64, torch.uint8])
def test_scaled_dot_product_attention_nonbool_mask(q, k, v, mask, mdtype):
    """A 0/1 integer mask means the same as the boolean one (nonzero = attend) on every path; the HIP kernel
    treats it so too (``ops/attention.py``)."""
    ref = run_scaled_dot_product_attention(q, k, v, mask)
    got = run_scaled_dot_product_attention(q, k, v, mask.to(mdtype))
    assert torch.equal(got, ref)


def test_scaled_dot_product_attention_float_mask_refused(q, k, v, mask):
    """A floating-point mask is ambiguous -- torch reads it as additive (0 = attend, -inf = block), the inverse of
    the nonzero-means-attend reading -- so it is refused instead of silently inverted."""
    with pytest.raises(TypeError, match="floating-point mask"):
        run_scaled_dot_product_attention(q, k, v, mask.to(torch.float32))


def test_rope(numpy_snapshot, in_embeddings, d_model, theta, n_queries, pos_ids):
    out = run_rope(d_model, theta, n_queries, in_embeddings, pos_ids)
    numpy_snapshot.assert_match(out, atol=1e-6)


def test_silu_matches_pytorch():
    x = torch.randn(5, 7)
    torch.testing.assert_close(run_silu(x), torch.nn.functional.silu(x), atol=1e-6, rtol=0)


# ---------------------------------------------------------------- snapshots needing the reference weights
def test_linear_snapshot(numpy_snapshot, ts_state_dict, in_embeddings, d_model, d_ff):
    w = ts_state_dict[0]["layers.0.ffn.w1.weight"]
    numpy_snapshot.assert_match(run_linear(d_model, d_ff, w, in_embeddings), test_name="test_linear")


def test_embedding_snapshot(numpy_snapshot, ts_state_dict, in_indices, vocab_size, d_model):
    w = ts_state_dict[0]["token_embeddings.weight"]
    numpy_snapshot.assert_match(run_embedding(vocab_size, d_model, w, in_indices), test_name="test_embedding")


def test_transformer_lm_snapshot(numpy_snapshot, ts_state_dict, in_indices, vocab_size, n_keys, d_model, n_layers,
                                 n_heads, d_ff, theta):
    sd, cfg = ts_state_dict
    out = run_transformer_lm(vocab_size, n_keys, d_model, n_layers, n_heads, d_ff, theta, sd, in_indices)
    numpy_snapshot.assert_match(out, atol=1e-4, rtol=1e-2, test_name="test_transformer_lm")
    out6 = run_transformer_lm(vocab_size, n_keys, d_model, n_layers, n_heads, d_ff, theta, sd, in_indices[:, :6])
    numpy_snapshot.assert_match(out6, atol=1e-4, rtol=1e-2, test_name="test_transformer_lm_truncated_input")


def test_swiglu_snapshot(numpy_snapshot, ts_state_dict, in_embeddings, d_model, d_ff):
    """``/root/reference/tests/test_model.py:43``."""
    w1, w2, w3 = (ts_state_dict[0][f"layers.0.ffn.{k}.weight"] for k in ("w1", "w2", "w3"))
    numpy_snapshot.assert_match(run_swiglu(d_model, d_ff, w1, w2, w3, in_embeddings), atol=1e-5,
                                test_name="test_swiglu")


def _attn_weights(sd):
    return [sd[f"layers.0.attn.{k}_proj.weight"] for k in ("q", "k", "v", "output")]


def test_multihead_self_attention_snapshot(numpy_snapshot, ts_state_dict, in_embeddings, d_model, n_heads):
    """``/root/reference/tests/test_model.py:77``."""
    out = run_multihead_self_attention(d_model, n_heads, *_attn_weights(ts_state_dict[0]), in_embeddings)
    numpy_snapshot.assert_match(out, atol=1e-6, test_name="test_multihead_self_attention")


def test_multihead_self_attention_with_rope_snapshot(numpy_snapshot, ts_state_dict, in_embeddings, d_model, n_heads,
                                                     n_keys, theta, pos_ids):
    """``/root/reference/tests/test_model.py:94`` (positions as a (1, seq) batch, as the reference passes them)."""
    out = run_multihead_self_attention_with_rope(d_model, n_heads, n_keys, theta, *_attn_weights(ts_state_dict[0]),
                                                 in_embeddings, pos_ids.reshape(1, -1))
    numpy_snapshot.assert_match(out, atol=1e-6, test_name="test_multihead_self_attention_with_rope")


def test_transformer_block_snapshot(numpy_snapshot, ts_state_dict, in_embeddings, d_model, n_heads, d_ff, n_keys,
                                    theta):
    """``/root/reference/tests/test_model.py:158``."""
    weights = {k.replace("layers.0.", ""): v for k, v in ts_state_dict[0].items() if "layers.0." in k}
    out = run_transformer_block(d_model, n_heads, d_ff, n_keys, theta, weights, in_embeddings)
    numpy_snapshot.assert_match(out, atol=1e-6, test_name="test_transformer_block")


def test_rmsnorm_snapshot(numpy_snapshot, ts_state_dict, in_embeddings):
    """``/root/reference/tests/test_model.py:176``."""
    w = ts_state_dict[0]["layers.1.ln1.weight"]
    numpy_snapshot.assert_match(run_rmsnorm(w.shape[0], 1e-5, w, in_embeddings), atol=1e-6, test_name="test_rmsnorm")


# ---------------------------------------------------------------- independent oracles
def _w(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) / math.sqrt(shape[-1])


def _oracle_rope(x, pos, theta):
    d = x.shape[-1]
    out = x.clone()
    for i in range(d // 2):
        ang = pos.double().unsqueeze(-1) * theta ** (-2 * i / d)
        c, s = torch.cos(ang).float().squeeze(-1), torch.sin(ang).float().squeeze(-1)
        a, b = x[..., 2 * i], x[..., 2 * i + 1]
        out[..., 2 * i] = a * c - b * s
        out[..., 2 * i + 1] = a * s + b * c
    return out


def _oracle_attn(x, wq, wk, wv, wo, H, theta=None):
    B, S, d = x.shape
    D = d // H
    q = torch.einsum("bsd,ed->bse", x, wq).view(B, S, H, D).permute(0, 2, 1, 3)
    k = torch.einsum("bsd,ed->bse", x, wk).view(B, S, H, D).permute(0, 2, 1, 3)
    v = torch.einsum("bsd,ed->bse", x, wv).view(B, S, H, D).permute(0, 2, 1, 3)
    if theta is not None:
        pos = torch.arange(S).view(1, 1, S)
        q, k = _oracle_rope(q, pos, theta), _oracle_rope(k, pos, theta)
    s = torch.einsum("bhqd,bhkd->bhqk", q, k) / math.sqrt(D)
    s = s + torch.triu(torch.full((S, S), float("-inf")), 1)
    o = torch.einsum("bhqk,bhkd->bhqd", torch.softmax(s, -1), v)
    return torch.einsum("bse,de->bsd", o.permute(0, 2, 1, 3).reshape(B, S, d), wo)


def _rms(x, g, eps=1e-5):
    return x / torch.sqrt((x * x).mean(-1, keepdim=True) + eps) * g


def _swiglu(x, w1, w2, w3):
    a = x @ w1.t()
    return (a * torch.sigmoid(a) * (x @ w3.t())) @ w2.t()


def test_linear_and_embedding_oracle(in_embeddings, in_indices):
    w = _w(128, 64)
    torch.testing.assert_close(run_linear(64, 128, w, in_embeddings), in_embeddings @ w.t())
    e = _w(10_000, 64, seed=1)
    torch.testing.assert_close(run_embedding(10_000, 64, e, in_indices), e[in_indices])


def test_rmsnorm_oracle(in_embeddings):
    g = 1 + 0.1 * _w(64)
    torch.testing.assert_close(run_rmsnorm(64, 1e-5, g, in_embeddings), _rms(in_embeddings, g), atol=1e-6, rtol=1e-5)


def test_swiglu_oracle(in_embeddings):
    w1, w2, w3 = _w(128, 64, seed=1), _w(64, 128, seed=2), _w(128, 64, seed=3)
    torch.testing.assert_close(run_swiglu(64, 128, w1, w2, w3, in_embeddings), _swiglu(in_embeddings, w1, w2, w3),
                               atol=1e-5, rtol=1e-4)


def test_mha_oracle(in_embeddings):
    ws = [_w(64, 64, seed=s) for s in range(4)]
    torch.testing.assert_close(run_multihead_self_attention(64, 4, *ws, in_embeddings),
                               _oracle_attn(in_embeddings, *ws, 4), atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(
        run_multihead_self_attention_with_rope(64, 4, 16, 10000.0, *ws, in_embeddings,
                                               torch.arange(12).unsqueeze(0)),
        _oracle_attn(in_embeddings, *ws, 4, theta=10000.0), atol=1e-5, rtol=1e-4)


def test_mha_is_causal(in_embeddings):
    ws = [_w(64, 64, seed=s) for s in range(4)]
    full = run_multihead_self_attention(64, 4, *ws, in_embeddings)
    head = run_multihead_self_attention(64, 4, *ws, in_embeddings[:, :5])
    torch.testing.assert_close(full[:, :5], head, atol=1e-6, rtol=1e-5)


def _block_weights(d=64, f=128, seed=0, prefix=""):
    names = {"attn.q_proj.weight": (d, d), "attn.k_proj.weight": (d, d), "attn.v_proj.weight": (d, d),
             "attn.output_proj.weight": (d, d), "ffn.w1.weight": (f, d), "ffn.w2.weight": (d, f),
             "ffn.w3.weight": (f, d)}
    w = {prefix + k: _w(*s, seed=seed + i) for i, (k, s) in enumerate(names.items())}
    w[prefix + "ln1.weight"] = 1 + 0.1 * _w(d, seed=seed + 50)
    w[prefix + "ln2.weight"] = 1 + 0.1 * _w(d, seed=seed + 51)
    return w


def _oracle_block(x, w, p=""):
    h = x + _oracle_attn(_rms(x, w[p + "ln1.weight"]), w[p + "attn.q_proj.weight"], w[p + "attn.k_proj.weight"],
                         w[p + "attn.v_proj.weight"], w[p + "attn.output_proj.weight"], 4, theta=10000.0)
    return h + _swiglu(_rms(h, w[p + "ln2.weight"]), w[p + "ffn.w1.weight"], w[p + "ffn.w2.weight"],
                       w[p + "ffn.w3.weight"])


def test_transformer_block_oracle(in_embeddings):
    w = _block_weights()
    torch.testing.assert_close(run_transformer_block(64, 4, 128, 16, 10000.0, w, in_embeddings),
                               _oracle_block(in_embeddings, w), atol=1e-5, rtol=1e-4)


def test_transformer_lm_oracle(in_indices):
    w = {}
    for layer in range(3):
        w.update(_block_weights(seed=100 * layer, prefix=f"layers.{layer}."))
    w["token_embeddings.weight"] = _w(10_000, 64, seed=7)
    w["ln_final.weight"] = 1 + 0.1 * _w(64, seed=8)
    w["lm_head.weight"] = _w(10_000, 64, seed=9)
    # torch.compile prefixes are accepted (reference conftest.py:201)
    w_compiled = {"_orig_mod." + k: v for k, v in w.items()}
    out = run_transformer_lm(10_000, 16, 64, 3, 4, 128, 10000.0, w_compiled, in_indices)
    x = w["token_embeddings.weight"][in_indices]
    for layer in range(3):
        x = _oracle_block(x, w, f"layers.{layer}.")
    exp = _rms(x, w["ln_final.weight"]) @ w["lm_head.weight"].t()
    torch.testing.assert_close(out, exp, atol=1e-4, rtol=1e-3)
    # causal: a truncated input reproduces the prefix logits
    out6 = run_transformer_lm(10_000, 16, 64, 3, 4, 128, 10000.0, w, in_indices[:, :6])
    torch.testing.assert_close(out6, out[:, :6], atol=1e-4, rtol=1e-3)
