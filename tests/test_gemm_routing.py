"""CPU tests of the weight-gradient routing decisions in ``ops/gemm.py`` (no kernel runs here; the kernels' numerics
are in tests/test_kernels_gpu.py)."""

from __future__ import annotations

import torch

from bpe_transformer.ops import gemm


def test_group_splits_fill_the_chip_at_gpt2_b128():
    """GPT-2 B 128 (131 072 tokens): the two per-layer groups -- W2 + [W1; W3] (24 + 48 tiles) and Wo + [Wq; Wk; Wv]
    (9 + 27) -- get a split count whose workgroups fill >= 98 % of their waves of 256 CUs, where the shapes alone
    ran 240-243 workgroups (profiles/bench/dw_stamps_r6.log)."""
    t = 131072
    for tiles, mn in ((72, 72 * 65536), (36, 36 * 65536)):
        s = gemm.choose_splits_group(tiles, t, mn)
        wgs = tiles * s
        waves = -(-wgs // 256)
        assert wgs / (waves * 256) >= 0.98, (tiles, s)
        assert (t // 64) // s >= 64  # long enough splits: the fixed per-workgroup cost stays a few percent


def test_group_splits_depend_on_shapes_only():
    a = gemm.choose_splits_group(528, 65536, 528 * 65536)
    b = gemm.choose_splits_group(528, 65536, 528 * 65536)
    assert a == b and 1 <= a <= 64


def test_group_falls_back_off_gpu_and_for_odd_shapes():
    t = 256
    dy = torch.zeros(t, 256, dtype=torch.bfloat16)
    x = torch.zeros(t, 512, dtype=torch.bfloat16)
    g = torch.zeros(256, 512, dtype=torch.bfloat16)
    assert not gemm._group_ok([(g, dy, x), (g, dy, x)])  # CPU tensors
    assert not gemm._group_ok([(g, dy, x)])  # one problem: the per-shape route
    # the fallback path accumulates through the per-shape routes (hipBLASLt-free CPU addmm here)
    dy = torch.randn(t, 256, dtype=torch.bfloat16)
    x = torch.randn(t, 512, dtype=torch.bfloat16)
    g1 = torch.zeros(256, 512, dtype=torch.bfloat16)
    g2 = torch.zeros(256, 512, dtype=torch.bfloat16)
    gemm.accumulate_weight_grads([(g1, dy, x), (g2, dy, x)])
    ref = dy.float().t() @ x.float()
    assert torch.allclose(g1.float(), ref, rtol=2e-2, atol=2e-1) and torch.equal(g1, g2)


def test_ppt_candidate_only_when_the_transpose_fits_32_bit_offsets():
    assert "ppt" in gemm._candidates(2304, 768, 131072)
    big = 2**31 // 256 + 64  # X^T's leading dimension T times 256 rows past 2^31
    cands = gemm._candidates(2304, 768, big - big % 64)
    assert "ppt" not in cands and "pp" in cands


def test_swiglu_forward_fusion_rule(monkeypatch):
    """The fused [W1;W3] + gate GEMM: d_model <= 1024 at any token count; wider only at >= 65 536 tokens per
    micro-batch (where the L2-aware tile order made it win, profiles/bench/ab_llama_swiglu_fwd_fused_r6.log); an
    explicit BPE_FUSE_SWIGLU_FWD_MAX_D cap replaces the rule."""
    from bpe_transformer.models import fused_block as fb

    def probe(t, d, f):
        x = torch.empty(t, d, device="meta", dtype=torch.bfloat16)
        return fb._fuse_swiglu_fwd(x, torch.empty(2 * f, d, device="meta", dtype=torch.bfloat16))

    monkeypatch.setattr(fb, "_FUSE_SWIGLU_FWD_MAX_D", 0)
    assert probe(131072, 768, 2048) and probe(512, 768, 2048)
    assert probe(65536, 2048, 5632) and not probe(16384, 2048, 5632)
    assert not probe(65536 + 64, 2048, 5632)  # tokens not a multiple of the 256-row tiles
    monkeypatch.setattr(fb, "_FUSE_SWIGLU_FWD_MAX_D", 1024)
    assert not probe(65536, 2048, 5632) and probe(256, 1024, 512)
