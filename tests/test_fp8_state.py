"""FP8 scaling-state bookkeeping (CPU: no kernels involved)."""

import pytest
import torch

from bpe_transformer.ops.fp8 import Fp8State, quantize_reference


def test_state_dict_roundtrip():
    a = Fp8State(8, "cpu", history=4)
    a.hist.uniform_()
    a.scale.fill_(16.0)
    a.inv_scale.fill_(1 / 16.0)
    a.pos = 5
    b = Fp8State(8, "cpu", history=4)
    b.load_state_dict(a.state_dict())
    assert torch.equal(b.hist, a.hist) and torch.equal(b.scale, a.scale) and b.pos == 5
    with pytest.raises(ValueError):
        Fp8State(4, "cpu", history=4).load_state_dict(a.state_dict())


def test_quantize_reference_saturates_and_rounds():
    x = torch.tensor([0.0, 1.0, -3.0, 1000.0, 0.1])
    y = quantize_reference(x, 1.0)
    assert y[3].item() == 448.0  # saturating cast
    assert y[1].item() == 1.0 and y[2].item() == -3.0
    assert abs(y[4].item() - 0.1) < 0.01  # e4m3: 3 mantissa bits


def test_model_enable_fp8_assigns_slots():
    from bpe_transformer.models import TransformerLM

    m = TransformerLM(100, 16, 32, 3, 2, 64)
    st = m.enable_fp8(history=8)
    assert st.n == 24 and st.hist.shape == (24, 8)
    assert [layer.fp8[1] for layer in m.layers] == [0, 8, 16]


def test_fp8_gemm_routing(monkeypatch):
    """BPE_FP8_GEMM routing (ops/fp8.py): the shipped table sends exactly its listed (M, N, K, A-format) shapes to
    the HIP fp8 kernel; "hip" / "lib" force one path."""
    import torch

    from bpe_transformer.ops import fp8

    assert (16384, 2560, 2048, "e4m3") in fp8._HIP_ROUTES
    monkeypatch.setattr(fp8, "_MODE", "routes")
    assert fp8._use_hip(16384, 2560, 2048, torch.float8_e4m3fn)
    assert not fp8._use_hip(16384, 2560, 2048, torch.float8_e5m2)  # same shape, other format: not measured
    assert not fp8._use_hip(16384, 2048, 2048, torch.float8_e4m3fn)
    monkeypatch.setattr(fp8, "_MODE", "hip")
    assert fp8._use_hip(16384, 2048, 2048, torch.float8_e4m3fn)
    monkeypatch.setattr(fp8, "_MODE", "lib")
    assert not fp8._use_hip(16384, 2560, 2048, torch.float8_e4m3fn)
