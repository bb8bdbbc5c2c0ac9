"""End-to-end GPU model tests: the fused bf16 HIP path vs the fp32 oracle model."""

from __future__ import annotations

import copy

import pytest
import torch

from bpe_transformer.models import TransformerLM

pytestmark = pytest.mark.gpu


def _pair(gpu_device, **kw):
    torch.manual_seed(0)
    cfg = dict(vocab_size=1000, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=512)
    cfg.update(kw)
    ref = TransformerLM(**cfg)
    gpu = copy.deepcopy(ref).to(gpu_device, torch.bfloat16)
    return ref, gpu


def test_forward_matches_oracle(gpu_device):
    ref, gpu = _pair(gpu_device)
    ids = torch.randint(0, 1000, (2, 128))
    lr = ref(ids)
    lg = gpu(ids.to(gpu_device)).float().cpu()
    err = (lg - lr).abs().max() / lr.abs().max()
    assert err < 5e-2, err


@pytest.mark.parametrize("heads", [4, 2])
def test_loss_and_grads_match_oracle(gpu_device, heads):
    """Head size 64 (4 heads) and 128 (2 heads: the D = 128 split backward, RoPE in the QKV GEMM epilogue)."""
    ref, gpu = _pair(gpu_device, num_heads=heads)
    ids = torch.randint(0, 1000, (2, 128))
    tgt = torch.randint(0, 1000, (2, 128))
    l_ref = ref.loss(ids, tgt)
    l_ref.backward()
    l_gpu = gpu.loss(ids.to(gpu_device), tgt.to(gpu_device))
    l_gpu.backward()
    assert abs(l_gpu.item() - l_ref.item()) < 3e-2
    for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
        e = (pg.grad.float().cpu() - pr.grad).norm() / pr.grad.norm().clamp_min(1e-12)
        assert e < 0.08, (n, float(e))


@pytest.mark.parametrize("fuse", [False, True])
def test_swiglu_forward_paths_match_oracle(gpu_device, monkeypatch, fuse):
    """Both SwiGLU forward paths of the fused block -- the gate in the [W1;W3] GEMM epilogue (gemm_swiglu_fwd,
    d_model <= 1024) and hipBLASLt + swiglu_fwd (wider models) -- against the fp32 oracle, with a batch whose
    token count (2 x 128) meets the fused kernel's 256-row tiles."""
    from bpe_transformer.models import fused_block

    monkeypatch.setattr(fused_block, "_FUSE_SWIGLU_FWD", fuse)
    probe = torch.empty(256, 256, device=gpu_device, dtype=torch.bfloat16)
    assert fused_block._fuse_swiglu_fwd(probe, torch.empty(1024, 256, device=gpu_device, dtype=torch.bfloat16)) == fuse
    ref, gpu = _pair(gpu_device)
    ids = torch.randint(0, 1000, (2, 128))
    tgt = torch.randint(0, 1000, (2, 128))
    l_ref = ref.loss(ids, tgt)
    l_ref.backward()
    l_gpu = gpu.loss(ids.to(gpu_device), tgt.to(gpu_device))
    l_gpu.backward()
    assert abs(l_gpu.item() - l_ref.item()) < 3e-2
    for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
        e = (pg.grad.float().cpu() - pr.grad).norm() / pr.grad.norm().clamp_min(1e-12)
        assert e < 0.08, (n, float(e))


def test_main_grad_path_matches_autograd(gpu_device):
    """Fused blocks accumulating into the flat buffer (main_grad) == per-parameter autograd grads."""
    from bpe_transformer.optim.flat import FlatParameters

    _, a = _pair(gpu_device)
    b = copy.deepcopy(a)
    flat = FlatParameters.from_module(a)
    for s in flat.slots:
        s.param.main_grad = flat.grad_view(s).view_as(s.param)
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    for _ in range(2):  # accumulation over two micro-batches
        a.loss(ids, tgt).backward()
        b.loss(ids, tgt).backward()
    for s, (n, pb) in zip(flat.slots, b.named_parameters()):
        ga = flat.grad_view(s).view_as(pb).float()
        e = (ga - pb.grad.float()).norm() / pb.grad.float().norm().clamp_min(1e-12)
        assert e < 1e-2, (n, float(e))


def test_grouped_dw_path_matches_per_shape_routes(gpu_device, monkeypatch):
    """The opt-in grouped weight-gradient launch (BPE_DW_GROUP=1: W2 + [W1; W3] and Wo + [Wq; Wk; Wv] dW in one
    split-K launch each, Wo's dW deferred past the attention backward) accumulates the same flat-buffer gradients as
    the per-shape routes, up to bf16 rounding of split-K partial sums in a different split count."""
    from bpe_transformer.ops import gemm
    from bpe_transformer.optim.flat import FlatParameters

    _, a = _pair(gpu_device)
    b = copy.deepcopy(a)
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    grads = []
    for model, group in ((a, True), (b, False)):
        monkeypatch.setattr(gemm, "_GROUP", group)
        flat = FlatParameters.from_module(model)
        for s in flat.slots:
            s.param.main_grad = flat.grad_view(s).view_as(s.param)
        model.loss(ids, tgt).backward()
        grads.append([flat.grad_view(s).float().clone() for s in flat.slots])
    assert gemm.groups_summary(), "the grouped launch did not run"
    for ga, gb in zip(*grads):
        assert torch.isfinite(ga).all()
        e = (ga - gb).norm() / gb.norm().clamp_min(1e-12)
        assert e < 1e-2, float(e)


def test_train_engine_reduces_loss(gpu_device):
    from bpe_transformer.train.engine import TrainEngine

    torch.manual_seed(0)
    model = TransformerLM(1000, 128, 256, 2, 4, 512, device=gpu_device, dtype=torch.bfloat16)
    eng = TrainEngine(model, lr=3e-3, weight_decay=0.0, max_grad_norm=1.0)
    x = torch.randint(0, 1000, (4, 128), device=gpu_device)
    y = torch.roll(x, -1, 1)
    first = eng.train_step([(x, y)]).item()
    for _ in range(30):
        last = eng.train_step([(x, y)]).item()
    assert last < first - 1.0, (first, last)


def test_generate(gpu_device):
    _, gpu = _pair(gpu_device)
    out = gpu.generate(torch.tensor([1, 2, 3], device=gpu_device), 8, temperature=0.0)
    assert out.shape == (11,)


@pytest.mark.parametrize("dgrad,wgrad", [(False, False), (True, False), (True, True)])
def test_fp8_close_to_bf16(gpu_device, dgrad, wgrad):
    """fp8 projections (e4m3 forward; with dgrad also e5m2 x e4m3 input gradients; with wgrad also e5m2 x e4m3
    weight gradients from the same gradient cast), delayed scaling: loss and grads stay close to the bf16 path
    after one calibration step."""
    _, a = _pair(gpu_device)
    b = copy.deepcopy(a)
    st = b.enable_fp8(dgrad=dgrad, wgrad=wgrad)
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    b.loss(ids, tgt).backward()  # calibration step: record activation / weight / gradient amaxes
    for s_ in b.fp8_states():
        s_.update()
    b.zero_grad()
    assert bool((st.scale > 1).all()), st.scale  # small activations/weights -> scales above 1
    if dgrad:
        assert bool((b.fp8_grad_state.scale > 1).all())  # gradients are far below the e5m2 range
    la = a.loss(ids, tgt)
    la.backward()
    lb = b.loss(ids, tgt)
    lb.backward()
    assert abs(la.item() - lb.item()) < 2e-2, (la.item(), lb.item())
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        e = (pb.grad.float() - pa.grad.float()).norm() / pa.grad.float().norm().clamp_min(1e-12)
        assert e < (0.2 if dgrad else 0.15), (n, float(e))


@pytest.mark.parametrize("flag", ["_FP8_SWIGLU_CAST", "_FP8_NORM_CAST", "_FP8_QKV_ROPE"])
def test_fp8_swiglu_cast_fused_matches_two_pass(gpu_device, monkeypatch, flag):
    """fp8 weight-gradient path: the SwiGLU gate and its backward (flag _FP8_SWIGLU_CAST), and the two RMSNorms
    (_FP8_NORM_CAST), writing only fp8 in both layouts give the loss and gradients of the two-pass form (bf16
    output, then the two-layout cast); the QKV projection with RoPE in the hand fp8 kernel's epilogue
    (_FP8_QKV_ROPE) those of the routed GEMM + rope_qk_."""
    from bpe_transformer.models import fused_block

    assert getattr(fused_block, flag)
    _, a = _pair(gpu_device)
    a.enable_fp8(dgrad=True, wgrad=True)
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    a.loss(ids, tgt).backward()  # calibration
    for s_ in a.fp8_states():
        s_.update()
    a.zero_grad()
    b = copy.deepcopy(a)
    la = a.loss(ids, tgt)
    la.backward()
    monkeypatch.setattr(fused_block, flag, False)
    lb = b.loss(ids, tgt)
    lb.backward()
    assert abs(la.item() - lb.item()) < 1e-3, (la.item(), lb.item())
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        e = (pb.grad.float() - pa.grad.float()).norm() / pa.grad.float().norm().clamp_min(1e-12)
        assert e < 2e-2, (n, float(e))


def test_fp8_fused_swiglu_gemms_match_separate_passes(gpu_device, monkeypatch):
    """fp8 weight-gradient path with the SwiGLU gate (and, opt-in, its backward) fused into the hand fp8 GEMMs'
    epilogues (ops/fp8.py matmul_swiglu / grads_swiglu) against the routed GEMMs + separate cast passes: the loss
    and every gradient agree (d_model 256, d_ff 512, 256 tokens: the shapes both fused kernels take)."""
    from bpe_transformer.ops import fp8 as F8

    monkeypatch.setattr(F8, "_SWIGLU_GEMM", True)
    monkeypatch.setattr(F8, "_SWIGLU_BWD_GEMM", True)
    _, a = _pair(gpu_device)
    a.enable_fp8(dgrad=True, wgrad=True)
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    a.loss(ids, tgt).backward()  # calibration
    for s_ in a.fp8_states():
        s_.update()
    a.zero_grad()
    b = copy.deepcopy(a)
    calls = {"fwd": 0, "bwd": 0}
    real_f, real_b = F8.swiglu_gemm_ok, F8.swiglu_bwd_gemm_ok

    def count(key, fn):
        def f(*args):
            ok = fn(*args)
            calls[key] += int(ok)
            return ok
        return f

    from bpe_transformer.models import fused_block
    monkeypatch.setattr(fused_block, "swiglu_gemm_ok", count("fwd", real_f))
    monkeypatch.setattr(fused_block, "swiglu_bwd_gemm_ok", count("bwd", real_b))
    la = a.loss(ids, tgt)
    la.backward()
    assert calls["fwd"] > 0 and calls["bwd"] > 0, calls
    monkeypatch.setattr(F8, "_SWIGLU_GEMM", False)
    monkeypatch.setattr(F8, "_SWIGLU_BWD_GEMM", False)
    lb = b.loss(ids, tgt)
    lb.backward()
    assert abs(la.item() - lb.item()) < 1e-2, (la.item(), lb.item())
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        e = (pb.grad.float() - pa.grad.float()).norm() / pa.grad.float().norm().clamp_min(1e-12)
        assert e < 5e-2, (n, float(e))


def test_fp8_engine_reduces_loss(gpu_device):
    from bpe_transformer.train.engine import TrainEngine

    torch.manual_seed(0)
    model = TransformerLM(1000, 128, 256, 2, 4, 512, device=gpu_device, dtype=torch.bfloat16)
    model.enable_fp8()
    eng = TrainEngine(model, lr=3e-3, weight_decay=0.0, max_grad_norm=1.0)
    x = torch.randint(0, 1000, (4, 128), device=gpu_device)
    y = torch.roll(x, -1, 1)
    first = eng.train_step([(x, y)]).item()
    for _ in range(30):
        last = eng.train_step([(x, y)]).item()
    assert last < first - 1.0, (first, last)
    assert model.fp8_state.pos == 31


def test_fp8_second_backward_raises(gpu_device):
    """The fp8 weight-gradient path frees the block's saved fp8 activations in its backward: a second backward through
    the same graph (retain_graph=True) raises a clear error instead of failing inside a GEMM on missing operands."""
    torch.manual_seed(0)
    model = TransformerLM(1000, 128, 256, 2, 4, 512, device=gpu_device, dtype=torch.bfloat16)
    model.enable_fp8(wgrad=True)
    x = torch.randint(0, 1000, (4, 128), device=gpu_device)
    loss = model.loss(x, torch.roll(x, -1, 1))
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="backward ran twice"):
        loss.backward()


@pytest.mark.parametrize("heads", [4, 2])
def test_forward_and_backward_are_bitwise_deterministic(gpu_device, heads):
    """Every kernel of the step is run-to-run deterministic at D = 64 and D = 128: the forward (attention, norms, CE,
    GEMM routing) and -- since the split attention backward has no dQ atomics (csrc/flash_attn_bwd_split.hip) and
    the split-K weight gradients reduce their fp32 slabs in a fixed order -- every gradient as well."""
    import torch.ops

    assert torch.ops.bpe_hip.fa_bwd_config(-1) == 0, "the default backward is the split form"
    assert not torch.ops.bpe_hip.fa_bwd_needs_dq_acc(256 // heads)
    _, gpu = _pair(gpu_device, num_heads=heads)
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    with torch.no_grad():
        a = gpu.loss(ids, tgt)
        b = gpu.loss(ids, tgt)
    assert torch.equal(a, b)
    grads = []
    for _ in range(2):
        gpu.zero_grad(set_to_none=True)
        gpu.loss(ids, tgt).backward()
        grads.append([p.grad.clone() for p in gpu.parameters()])
    for (n, _), g0, g1 in zip(gpu.named_parameters(), *grads):
        assert torch.equal(g0, g1), n


def test_engine_phase_timing(gpu_device):
    from bpe_transformer.train.engine import TrainEngine

    torch.manual_seed(0)
    model = TransformerLM(1000, 128, 256, 2, 4, 512, device=gpu_device, dtype=torch.bfloat16)
    eng = TrainEngine(model, time_phases=True)
    x = torch.randint(0, 1000, (4, 128), device=gpu_device)
    for _ in range(3):
        eng.train_step([(x, torch.roll(x, -1, 1))])
    ph = eng.phase_times()
    assert set(ph) == {"fwd_ms", "bwd_ms", "comm_ms", "opt_ms"} and all(v >= 0 for v in ph.values())


def test_padded_lm_head_matches_unpadded(gpu_device):
    """The zero-row padded LM head (vocab 1000 -> 1024 rows in the flat buffer) gives the same loss and
    gradients as the unpadded head, and AdamW keeps the pad rows exactly zero."""
    from bpe_transformer.train.engine import TrainEngine

    _, a = _pair(gpu_device)
    b = copy.deepcopy(a)
    b.lm_head.pad_rows = None
    ea = TrainEngine(a, lr=1e-3, weight_decay=0.1, max_grad_norm=None)
    eb = TrainEngine(b, lr=1e-3, weight_decay=0.1, max_grad_norm=None)
    wp = a.lm_head.weight._bpe_padded
    assert wp.shape == (1024, 256) and not hasattr(b.lm_head.weight, "_bpe_padded")
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    for _ in range(3):
        la = ea.train_step([(ids, tgt)])
        lb = eb.train_step([(ids, tgt)])
        assert abs(la.item() - lb.item()) < 1e-3, (la.item(), lb.item())
    ga, gb = a.lm_head.weight._bpe_padded_grad, b.lm_head.weight.grad
    assert torch.count_nonzero(ga[1000:]) == 0 and torch.count_nonzero(wp[1000:]) == 0
    e = (ga[:1000].float() - gb.float()).norm() / gb.float().norm()
    assert e < 1e-2, float(e)


def test_streamed_lm_head_trains_like_logits_mode(gpu_device):
    """lm_head_mode "streamed" (dh / dW formed chunk by chunk in the forward, no full logits buffer; ops/loss.py)
    through the training engine tracks the default logits mode step for step, padded head included."""
    from bpe_transformer.train.engine import TrainEngine

    _, a = _pair(gpu_device)
    b = copy.deepcopy(a)
    b.lm_head_mode, b.lm_head_chunk = "streamed", 96  # 256 tokens -> chunks 96, 96, 64
    ea = TrainEngine(a, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0)
    eb = TrainEngine(b, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0)
    ids = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt = torch.randint(0, 1000, (2, 128), device=gpu_device)
    tgt[0, ::5] = -100
    for _ in range(4):
        la = ea.train_step([(ids, tgt)])
        lb = eb.train_step([(ids, tgt)])
        assert abs(la.item() - lb.item()) < 5e-3, (la.item(), lb.item())
    assert torch.count_nonzero(b.lm_head.weight._bpe_padded[1000:]) == 0
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        e = (pa.float() - pb.float()).norm() / pa.float().norm()
        assert e < 1e-2, (n, float(e))
