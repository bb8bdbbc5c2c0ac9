"""gfx950 HIP kernels vs plain-PyTorch fp32 references (forward AND backward).

Every test here runs the hand-written kernel (``torch.ops.bpe_hip.*``) on the
GPU and compares it against the same op computed in fp32 by the oracle in
``bpe_transformer.ops.reference`` from the SAME (rounded) inputs.
"""

from __future__ import annotations

import math

import pytest
import torch

from bpe_transformer import ops
from bpe_transformer.ops import reference as R

pytestmark = pytest.mark.gpu


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def _ref_grads(fn, inputs, dout):
    xs = [x.detach().float().cpu().requires_grad_(True) for x in inputs]
    y = fn(*xs)
    y.backward(dout.float().cpu())
    return y.detach(), [x.grad for x in xs]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
# (64, 768), (4096, 768), (6, 1024) bf16 and (10, 384) fp32: the half-wave-row backward (csrc/rmsnorm.hip), the
# second with a grid-stride loop over more rows than one round; (7, 512): odd rows, the one-wave-per-row kernel
@pytest.mark.parametrize("shape", [(64, 768), (3, 5, 2048), (7, 512), (2048, 2048), (33, 4096), (4096, 768), (6, 1024),
                                   (10, 384)])
def test_rmsnorm(gpu_device, dtype, shape):
    torch.manual_seed(0)
    x = torch.randn(*shape, device=gpu_device, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(shape[-1], device=gpu_device, dtype=dtype)).requires_grad_(True)
    y = ops.rmsnorm(x, w, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr, (gx, gw) = _ref_grads(lambda a, b: R.rmsnorm(a, b, 1e-5), [x, w], dy)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(y.cpu(), yr) < tol
    assert rel(x.grad.cpu(), gx) < tol * 2
    assert rel(w.grad.cpu(), gw) < tol * 2


@pytest.mark.parametrize("M,N", [(4096, 768), (64, 512), (7, 768)])
def test_rmsnorm_bwd_residual_grad(gpu_device, M, N):
    """rmsnorm_bwd with the residual-branch gradient fused in: dx(dres) == dx + dres and dw unchanged."""
    torch.manual_seed(2)
    h = torch.ops.bpe_hip
    x = torch.randn(M, N, device=gpu_device, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(N, device=gpu_device)).to(torch.bfloat16)
    _, rstd = h.rmsnorm_fwd(x, w, 1e-5)
    dy = torch.randn_like(x)
    dres = torch.randn_like(x)
    dx0, dw0 = h.rmsnorm_bwd(dy, x, w, rstd, None)
    dx1, dw1 = h.rmsnorm_bwd(dy, x, w, rstd, dres)
    assert torch.equal(dw0, dw1)
    assert rel(dx1.float(), dx0.float() + dres.float()) < 1e-2
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    R.rmsnorm(xr, wr, 1e-5).backward(dy.float())
    assert rel(dx0.float(), xr.grad) < 2e-2 and rel(dw0.float(), wr.grad) < 2e-2
    # dw added straight into a gradient slot (bf16 / fp32): slot + the fp32 column sums, rounded once
    for dt in (torch.bfloat16, torch.float32):
        slot = torch.randn(N, device=gpu_device).to(dt)
        before = slot.float().clone()
        dx2, dw2 = h.rmsnorm_bwd(dy, x, w, rstd, dres, slot)
        assert dw2.numel() == 0 and torch.equal(dx2, dx1)
        if dt == torch.bfloat16:
            assert rel(slot.float(), before + dw0.float()) < 1e-2
        else:  # fp32: the column sums are added unrounded (dw0 is their bf16 rounding)
            assert rel(slot - before, wr.grad) < 2e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_swiglu_gate(gpu_device, dtype):
    torch.manual_seed(0)
    gu = torch.randn(33, 2 * 256, device=gpu_device, dtype=dtype, requires_grad=True)
    a = ops.swiglu_gate(gu)
    d = torch.randn_like(a)
    a.backward(d)
    ar, (g,) = _ref_grads(lambda t: R.silu(t[:, :256]) * t[:, 256:], [gu], d)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(a.cpu(), ar) < tol
    assert rel(gu.grad.cpu(), g) < tol * 2


@pytest.mark.parametrize("kind", ["silu", "gelu"])
def test_activations(gpu_device, kind):
    torch.manual_seed(0)
    x = (4 * torch.randn(1024, device=gpu_device)).requires_grad_(True)
    f = ops.silu if kind == "silu" else ops.gelu
    fr = R.silu if kind == "silu" else R.gelu_tanh
    y = f(x)
    d = torch.randn_like(y)
    y.backward(d)
    yr, (g,) = _ref_grads(fr, [x], d)
    assert rel(y.cpu(), yr) < 1e-5
    assert rel(x.grad.cpu(), g) < 1e-4
    # overflow-safe tanh: the reference Triton kernel returns NaN here
    big = torch.tensor([100.0, 1e4, -1e4], device=gpu_device)
    assert torch.isfinite(ops.gelu(big)).all()


@pytest.mark.parametrize("V", [50257, 1000, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cross_entropy(gpu_device, V, dtype):
    torch.manual_seed(0)
    x = torch.randn(37, V, device=gpu_device, dtype=dtype, requires_grad=True)
    t = torch.randint(0, V, (37,), device=gpu_device)
    loss = ops.cross_entropy(x, t)
    loss.backward()
    xr = x.detach().float().cpu().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(xr, t.cpu())
    lr_.backward()
    assert abs(loss.item() - lr_.item()) < (1e-5 if dtype == torch.float32 else 2e-2)
    assert rel(x.grad.cpu(), xr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)
    # large-logit stability (tests/test_nn_utils.py:53 in the reference)
    big = 1000.0 * torch.rand(8, 5, device=gpu_device)
    tb = torch.randint(0, 5, (8,), device=gpu_device)
    ref = torch.nn.functional.cross_entropy(big.cpu(), tb.cpu())
    assert abs(ops.cross_entropy(big, tb).item() - ref.item()) < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cross_entropy_target_positions(gpu_device, dtype):
    """Targets in the unaligned head, the body and the scalar tail of odd-length rows (V = 50257: row r starts at
    element 50257 r), and ignored rows: the register kernel writes softmax * scale everywhere and stores the target's
    "- scale" once per row after the row's other stores."""
    V = 50257
    torch.manual_seed(5)
    x = torch.randn(24, V, device=gpu_device, dtype=dtype, requires_grad=True)
    t = torch.tensor([0, 1, 2, 3, 5, 7, 8, 9, 15, 16, 4000, 25000, V - 9, V - 8, V - 7, V - 2, V - 1,
                      -100, 6, V - 3, 12345, -100, 31, 63], device=gpu_device)
    loss = ops.cross_entropy(x, t)
    loss.backward()
    xr = x.detach().float().cpu().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(xr, t.cpu(), ignore_index=-100)
    lr_.backward()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert abs(loss.item() - lr_.item()) < tol
    assert rel(x.grad.cpu(), xr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)
    g, gr = x.grad.float().cpu(), xr.grad
    rows = torch.arange(24)
    ok = t.cpu() != -100
    # the target entries themselves (negative: p - 1), and the ignored rows all zero
    assert torch.allclose(g[rows[ok], t.cpu()[ok]], gr[rows[ok], t.cpu()[ok]], rtol=2e-2, atol=1e-6)
    assert g[~ok].abs().max().item() == 0.0


def test_cross_entropy_ignore_index(gpu_device):
    torch.manual_seed(0)
    x = torch.randn(16, 100, device=gpu_device, requires_grad=True)
    t = torch.randint(0, 100, (16,), device=gpu_device)
    t[::3] = -100
    loss = ops.cross_entropy(x, t)
    loss.backward()
    xr = x.detach().cpu().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(xr, t.cpu(), ignore_index=-100)
    lr_.backward()
    assert abs(loss.item() - lr_.item()) < 1e-5
    assert rel(x.grad.cpu(), xr.grad) < 1e-4


def test_lm_head_cross_entropy(gpu_device):
    torch.manual_seed(0)
    h = torch.randn(64, 256, device=gpu_device, dtype=torch.bfloat16, requires_grad=True)
    w = (0.05 * torch.randn(50257, 256, device=gpu_device, dtype=torch.bfloat16)).requires_grad_(True)
    t = torch.randint(0, 50257, (64,), device=gpu_device)
    loss = ops.lm_head_cross_entropy(h, w, t)
    (2.0 * loss).backward()
    hr = h.detach().float().cpu().requires_grad_(True)
    wr = w.detach().float().cpu().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(hr @ wr.t(), t.cpu())
    (2.0 * lr_).backward()
    assert abs(loss.item() - lr_.item()) < 2e-2
    assert rel(h.grad.cpu(), hr.grad) < 3e-2
    assert rel(w.grad.cpu(), wr.grad) < 3e-2


@pytest.mark.parametrize("mode,chunk", [("logits", 384), ("streamed", 384), ("streamed", 4096)])
def test_lm_head_ce_chunked_matches_one_pass(gpu_device, mode, chunk):
    """Token-chunked LM head + CE (the logits mode's chunks, or the streamed mode that forms dh / dW in the forward
    and never holds the full logits) == one pass: M not a multiple of the chunk, ignore_index rows, the
    row-padded vocab weight from the flat buffer, and the LM-head dW accumulated in place into the flat gradient."""
    from bpe_transformer.optim import FlatParameters

    V, d, M = 5003, 256, 1000
    torch.manual_seed(0)
    head = torch.nn.Linear(d, V, bias=False).to(gpu_device, torch.bfloat16)
    head.pad_rows = (V + 255) // 256 * 256
    flat = FlatParameters.from_module(head)
    assert head.weight._bpe_padded.shape[0] == head.pad_rows
    h0 = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    t = torch.randint(0, V, (M,), device=gpu_device)
    t[::7] = -100
    out = {}
    for key, (md, ck) in {"one": ("logits", 0), "chunked": (mode, chunk)}.items():
        flat.zero_grad()
        h = h0.clone().requires_grad_(True)
        loss = ops.lm_head_cross_entropy(h, head.weight, t, chunk=ck, mode=md)
        (3.0 * loss).backward()
        torch.cuda.synchronize()
        out[key] = (loss.detach().float(), h.grad.float(), flat.grad.float().clone())
    (l0, dh0, g0), (l1, dh1, g1) = out["one"], out["chunked"]
    # same math; only the library GEMM's per-chunk kernel choice (rounding of the bf16 logits) may differ
    assert abs(l0.item() - l1.item()) < 1e-3
    assert rel(dh1, dh0) < 1e-2
    assert rel(g1, g0) < 1e-2
    assert float(g0.view(-1)[V * d :].abs().max()) == 0.0  # pad rows get no gradient
    hr = h0.float().cpu().requires_grad_(True)
    wr = head.weight.detach().float().cpu().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(hr @ wr.t(), t.cpu(), ignore_index=-100)
    (3.0 * lr_).backward()
    assert abs(l1.item() - lr_.item()) < 2e-2
    assert rel(dh1.cpu(), hr.grad) < 3e-2
    assert rel(g1[: V * d].view(V, d).cpu(), wr.grad) < 3e-2


@pytest.mark.parametrize("mode", ["logits", "streamed"])
def test_lm_head_ce_no_grad_is_loss_only(gpu_device, mode):
    """Without a backward (no_grad, or nothing requiring grad) the LM head + CE takes the loss-only path: the loss
    equals the training path's, no dh / dW work runs (the weight's flat gradient stays untouched) and the largest
    temporary is one [chunk, vocab] buffer, not the full logits."""
    V, d, M = 5003, 256, 3000
    torch.manual_seed(4)
    w = (0.05 * torch.randn(V, d, device=gpu_device)).to(torch.bfloat16).requires_grad_(True)
    h0 = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    t = torch.randint(0, V, (M,), device=gpu_device)
    t[::5] = -100
    ref = ops.lm_head_cross_entropy(h0.clone().requires_grad_(True), w, t, mode=mode).item()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    with torch.no_grad():
        got = ops.lm_head_cross_entropy(h0, w, t, mode=mode, chunk=1024).item()
    peak = torch.cuda.max_memory_allocated() - base
    assert abs(got - ref) < 1e-3, (got, ref)
    assert w.grad is None
    assert peak < 1024 * V * 2 * 1.5, peak  # one chunk buffer (+ small temporaries), never M x V


def test_transpose_bf16_scaled(gpu_device):
    """The transposed copy with a device scale (the LM head's upstream gradient folded in): bf16(scale * W)^T
    bitwise, and plain W^T without it."""
    torch.manual_seed(8)
    w = torch.randn(192, 320, device=gpu_device, dtype=torch.bfloat16)
    sc = torch.tensor([0.37], device=gpu_device)
    h = torch.ops.bpe_hip
    assert torch.equal(h.transpose_bf16(w), w.t().contiguous())
    assert torch.equal(h.transpose_bf16(w, sc), (w.float() * 0.37).to(torch.bfloat16).t().contiguous())


def test_weight_grad_x_scale_on_the_ppt_route(gpu_device):
    """accumulate_weight_grad's x_scale on the ppt route (applied in the X^T copy) == the route on a pre-scaled X,
    bitwise; and the other routes scale X first."""
    from bpe_transformer.ops.gemm import _run

    torch.manual_seed(9)
    n, k, t = 512, 256, 2048
    dy = torch.randn(t, n, device=gpu_device, dtype=torch.bfloat16)
    x = torch.randn(t, k, device=gpu_device, dtype=torch.bfloat16)
    sc = torch.tensor(0.5, device=gpu_device)  # the autograd scalar as the LM head sees it (0-dim)
    xs = (x.float() * 0.5).to(torch.bfloat16)
    for route in ("ppt", "pp", "blas"):
        g1 = torch.zeros(n, k, device=gpu_device, dtype=torch.bfloat16)
        g2 = torch.zeros_like(g1)
        _run(route, g1, dy, x, sc)
        _run(route, g2, dy, xs)
        assert torch.equal(g1, g2), route


def test_lm_head_dx_tn_matches_nn(gpu_device, monkeypatch):
    """The LM-head input gradient through the transposed weight copy (hipBLASLt TN layout, the default) equals
    the NN call on the stored weight up to GEMM rounding, and both match the fp32 oracle."""
    from bpe_transformer.ops import loss as L

    V, d, M = 4096, 256, 512  # V, d multiples of 64: the TN path applies
    torch.manual_seed(3)
    w = (0.05 * torch.randn(V, d, device=gpu_device)).to(torch.bfloat16)
    h0 = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    t = torch.randint(0, V, (M,), device=gpu_device)
    dh = {}
    for tn in (False, True):
        monkeypatch.setattr(L, "_HEAD_DX_TN", tn)
        h = h0.clone().requires_grad_(True)
        ops.lm_head_cross_entropy(h, w, t).backward()
        dh[tn] = h.grad.float()
    assert rel(dh[True], dh[False]) < 1e-2
    hr = h0.float().cpu().requires_grad_(True)
    torch.nn.functional.cross_entropy(hr @ w.float().cpu().t(), t.cpu()).backward()
    assert rel(dh[True].cpu(), hr.grad) < 3e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_embedding(gpu_device, dtype):
    torch.manual_seed(0)
    W = torch.randn(1000, 768, device=gpu_device, dtype=dtype, requires_grad=True)
    ids = torch.randint(0, 50, (4, 300), device=gpu_device)  # many repeats
    y = ops.embedding(W, ids)
    d = torch.randn_like(y)
    y.backward(d)
    Wr = W.detach().float().cpu().requires_grad_(True)
    yr = Wr[ids.cpu()]
    yr.backward(d.float().cpu())
    assert torch.equal(y.float().cpu(), yr.detach())
    assert rel(W.grad.cpu(), Wr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)
    # deterministic: a second backward gives bitwise-identical gradients
    g1 = W.grad.clone()
    W.grad = None
    ops.embedding(W, ids).backward(d)
    assert torch.equal(W.grad, g1)


def test_softmax(gpu_device):
    x = torch.tensor([[0.4655, 0.8303, 0.9608, 0.9656, 0.6840], [0.2583, 0.2198, 0.9334, 0.2995, 0.1722]],
                     device=gpu_device)
    exp = torch.softmax(x.cpu(), -1)
    assert torch.allclose(ops.softmax(x, -1).cpu(), exp, atol=1e-6)
    assert torch.allclose(ops.softmax(x + 100, -1).cpu(), exp, atol=1e-6)
    z = torch.randn(3, 7, 11, device=gpu_device, requires_grad=True)
    y = ops.softmax(z, dim=1)
    d = torch.randn_like(y)
    y.backward(d)
    zr = z.detach().cpu().requires_grad_(True)
    yr = torch.softmax(zr, 1)
    yr.backward(d.cpu())
    assert rel(y.cpu(), yr.detach()) < 1e-5 and rel(z.grad.cpu(), zr.grad) < 1e-4


def test_rope(gpu_device):
    torch.manual_seed(0)
    cos, sin = R.rope_tables(64, 512, 10000.0, device=gpu_device)
    x = torch.randn(2, 4, 100, 64, device=gpu_device, requires_grad=True)
    pos = torch.randint(0, 512, (2, 1, 100), device=gpu_device)
    y = ops.apply_rope(x, cos, sin, pos)
    d = torch.randn_like(y)
    y.backward(d)
    yr, (g,) = _ref_grads(lambda t: R.apply_rope(t, cos.cpu(), sin.cpu(), pos.cpu()), [x], d)
    assert rel(y.cpu(), yr) < 1e-5 and rel(x.grad.cpu(), g) < 1e-5


def test_adamw_matches_torch(gpu_device):
    from bpe_transformer.optim import AdamW

    torch.manual_seed(0)
    p1 = torch.randn(1001, device=gpu_device, requires_grad=True)
    p2 = p1.detach().clone().requires_grad_(True)
    o1 = AdamW([p1], lr=1e-2, weight_decay=0.1, betas=(0.9, 0.95), eps=1e-8)
    o2 = torch.optim.AdamW([p2], lr=1e-2, weight_decay=0.1, betas=(0.9, 0.95), eps=1e-8)
    for _ in range(20):
        g = torch.randn_like(p1)
        p1.grad = g.clone()
        p2.grad = g.clone()
        o1.step()
        o2.step()
    assert rel(p1.detach(), p2.detach()) < 1e-5


@pytest.mark.parametrize("n,gdtype", [(1_000_005, torch.bfloat16), (4099, torch.float32), (7, torch.bfloat16)])
def test_fused_adamw_kernel_vs_cpu(gpu_device, n, gdtype):
    """The 8-wide AdamW kernel (ragged tail < 8, bf16 or fp32 gradients, clip coefficient, bf16 copy-out) vs
    the same update computed by the CPU path of ops.fused_adamw_step."""
    from bpe_transformer.ops.optim import fused_adamw_step

    torch.manual_seed(2)
    p = torch.randn(n)
    m = 0.1 * torch.randn(n)
    v = 0.01 * torch.rand(n)
    g = torch.randn(n).to(gdtype)
    scale = torch.tensor(0.5)
    ref = [t.clone() for t in (p, m, v)]
    fused_adamw_step(*ref, g, None, 1e-3, 0.9, 0.95, 1e-8, 0.1, 3, scale)
    gp, gm, gv = (t.to(gpu_device) for t in (p, m, v))
    out = torch.empty(n, device=gpu_device, dtype=torch.bfloat16)
    fused_adamw_step(gp, gm, gv, g.to(gpu_device), out, 1e-3, 0.9, 0.95, 1e-8, 0.1, 3, scale.to(gpu_device))
    for a, b in zip((gp, gm, gv), ref):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=1e-7)
    assert torch.equal(out.cpu(), gp.cpu().to(torch.bfloat16))


def test_flat_adamw_one_launch_matches_segments(gpu_device):
    """The masked single-launch AdamW (one byte per 64 elements selects weight decay) equals the per-segment
    launches bitwise over a model with decayed matrices and undecayed norm gains, three steps."""
    from bpe_transformer.models import TransformerLM
    from bpe_transformer.optim import FlatAdamW, FlatParameters

    res = []
    for masked in (True, False):
        torch.manual_seed(0)
        m = TransformerLM(300, 64, 64, 2, 4, 128, device=gpu_device, dtype=torch.bfloat16)
        flat = FlatParameters.from_module(m)
        opt = FlatAdamW(flat, lr=1e-2, weight_decay=0.1)
        assert opt.wd_mask is not None and len(opt.segments) > 2
        if not masked:
            opt.wd_mask = None
        g = torch.Generator(device="cpu").manual_seed(1)
        for _ in range(3):
            flat.grad.copy_(torch.randn(flat.grad.shape, generator=g).to(flat.grad.dtype))
            opt.step()
        res.append(opt.master.clone())
    assert torch.equal(res[0], res[1])


def test_flat_adamw_bf16_master(gpu_device):
    from bpe_transformer.optim import FlatAdamW, FlatParameters

    torch.manual_seed(0)
    lin = torch.nn.Linear(64, 33, bias=True).to(gpu_device, torch.bfloat16)
    ref = [p.detach().float().clone().requires_grad_(True) for p in lin.parameters()]
    flat = FlatParameters.from_module(lin)
    opt = FlatAdamW(flat, lr=1e-3, weight_decay=0.0)
    oref = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.0)
    for _ in range(5):
        flat.zero_grad()
        for p, r in zip(lin.parameters(), ref):
            g = torch.randn_like(r)
            p.grad.copy_(g.to(torch.bfloat16))
            r.grad = g.to(torch.bfloat16).float()
        opt.step()
        oref.step()
    for p, r in zip(lin.parameters(), ref):
        assert rel(p.detach(), r.detach().to(torch.bfloat16)) < 1e-2


def test_flat_adamw_skip_keeps_bias_correction(gpu_device):
    """HIP path: a skipped non-finite step does not advance the device step counter (bias correction), so the
    run with an inf gradient in the middle ends at the same weights as the run without it (vs the CPU path)."""
    from .test_trainer import _flat_opt_run

    opt, flat = _flat_opt_run(gpu_device, skip_at=1)
    ref, fref = _flat_opt_run(gpu_device)
    cpu, fcpu = _flat_opt_run("cpu")
    assert opt.calls == 5 and opt.step_count == 4
    assert torch.equal(flat.data, fref.data)
    torch.testing.assert_close(flat.data.cpu(), fcpu.data, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dtype,n", [(torch.float32, 9_000_003), (torch.bfloat16, 20_000_001)])
def test_grad_norm_large(gpu_device, dtype, n):
    """Sizes past two grid strides (2048 blocks x 256 threads x one vector each), with a ragged tail."""
    torch.manual_seed(1)
    ts = [torch.randn(n, device=gpu_device).to(dtype), torch.randn(77, device=gpu_device).to(dtype)]
    norm, _ = ops.grad_norm(ts, 1.0)
    exp = torch.sqrt(sum((t.double() ** 2).sum() for t in ts)).item()
    assert abs(norm.item() - exp) / exp < 1e-4


def test_grad_norm_clip(gpu_device):
    torch.manual_seed(0)
    ts = [torch.randn(n, device=gpu_device) for n in (5, 1000, 3333)]
    norm, coef = ops.grad_norm(ts, 1.0)
    exp = torch.sqrt(sum((t.cpu() ** 2).sum() for t in ts))
    assert abs(norm.item() - exp.item()) / exp.item() < 1e-5
    assert abs(coef.item() - 1.0 / (exp.item() + 1e-6)) < 1e-6
    params = [torch.nn.Parameter(t.clone()) for t in ts]
    refs = [torch.nn.Parameter(t.cpu().clone()) for t in ts]
    for p, r in zip(params, refs):
        p.grad = p.detach().clone()
        r.grad = r.detach().clone()
    ops.clip_grad_norm_(params, 1e-2)
    torch.nn.utils.clip_grad_norm_(refs, 1e-2)
    for p, r in zip(params, refs):
        assert rel(p.grad.cpu(), r.grad) < 1e-5


# ---------------------------------------------------------------- GEMM
@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("splits", [1, 4, 7])
@pytest.mark.parametrize("tile", [128, 256])
def test_gemm_layouts(gpu_device, a_k, b_k, splits, tile):
    if tile == 256 and (a_k or b_k):
        pytest.skip("the 256-tile kernel serves the weight-gradient (token-major) layout only")
    torch.manual_seed(0)
    Mo, No, R = (256, 384, 1024) if tile == 128 else (512, 768, 1536)
    A = torch.randn(Mo, R, device=gpu_device, dtype=torch.bfloat16)
    B = torch.randn(No, R, device=gpu_device, dtype=torch.bfloat16)
    Am = A if a_k else A.t().contiguous()
    Bm = B if b_k else B.t().contiguous()
    C = torch.randn(Mo, No, device=gpu_device, dtype=torch.bfloat16)
    ref = C.float() * 0.5 + A.float() @ B.float().t()
    torch.ops.bpe_hip.gemm(Am, a_k, Bm, b_k, C, 0.5, splits, tile)
    assert rel(C.cpu(), ref.cpu()) < 1e-2


@pytest.mark.parametrize("shape", [(64, 64), (2304, 768), (768, 4096), (192, 320)])
def test_transpose_bf16(gpu_device, shape):
    """LDS-tiled transpose (dX in the TN layout): exact, including a row-strided (sliced) input."""
    torch.manual_seed(3)
    R, C = shape
    big = torch.randn(R, C + 64, device=gpu_device, dtype=torch.bfloat16)
    for w in (big[:, :C].contiguous(), big[:, 64:]):
        t = torch.ops.bpe_hip.transpose_bf16(w)
        assert t.shape == (C, R) and t.is_contiguous()
        assert torch.equal(t.cpu(), w.t().cpu())


@pytest.fixture(params=[0, 1, 3], ids=["tile", "persist", "persist3"])
def gpp_mode(request, gpu_device):
    """gemm_pp kernel form: one tile per workgroup, persistent (one workgroup per CU), persistent with 3
    workgroups (several tiles each, unevenly split, even on small shapes)."""
    h = torch.ops.bpe_hip
    prev = h.gpp_persist_config(request.param)
    yield request.param
    h.gpp_persist_config(prev)


def test_gemm_swiglu_bwd(gpu_device, gpp_mode):
    """dY @ W2 with the SwiGLU backward in the epilogue vs the fp32 oracle of the same two steps."""
    torch.manual_seed(2)
    M, d, F = 512, 192, 768
    dy = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    w2 = (0.1 * torch.randn(d, F, device=gpu_device)).to(torch.bfloat16)
    gu = torch.randn(M, 2 * F, device=gpu_device, dtype=torch.bfloat16)
    dgu = torch.ops.bpe_hip.gemm_swiglu_bwd(dy, w2, gu)
    da = (dy.float() @ w2.float()).to(torch.bfloat16).float()  # the kernel rounds da to bf16 like the unfused path
    g, u = gu.float()[:, :F], gu.float()[:, F:]
    s = torch.sigmoid(g)
    ref = torch.cat([da * u * s * (1 + g * (1 - s)), da * g * s], 1)
    assert rel(dgu.cpu(), ref.cpu()) < 2e-2
    unfused = torch.ops.bpe_hip.swiglu_bwd((dy @ w2).contiguous(), gu)
    assert rel(dgu.cpu(), unfused.cpu()) < 2e-2


def test_gemm_swiglu_bwd_bitwise_on_exact_products(gpu_device, gpp_mode):
    """Small-integer dY and W2 make da = dY W2 exact (and exact in bf16), so the fused epilogue (packed two-element
    fp32 arithmetic, BPE_GPP_PK=1) must give bitwise the unfused ``swiglu_bwd`` of that da on the same gu."""
    torch.manual_seed(6)
    M, d, F = 512, 192, 768
    dy = torch.randint(-2, 3, (M, d), device=gpu_device).to(torch.bfloat16)
    w2 = torch.randint(-1, 2, (d, F), device=gpu_device).to(torch.bfloat16)
    gu = torch.randn(M, 2 * F, device=gpu_device, dtype=torch.bfloat16)
    da = (dy.float() @ w2.float()).to(torch.bfloat16)
    assert torch.equal(da.float(), dy.float() @ w2.float())  # exact
    dgu = torch.ops.bpe_hip.gemm_swiglu_bwd(dy, w2, gu)
    assert torch.equal(dgu, torch.ops.bpe_hip.swiglu_bwd(da.contiguous(), gu))


@pytest.mark.parametrize("M,d,F", [(512, 192, 768), (256, 64, 128), (512, 2048, 5632)])  # + Llama-1.1B width
def test_gemm_swiglu_fwd(gpu_device, gpp_mode, M, d, F):
    """x @ [W1; W3]^T with a = silu(g) * u in the epilogue.  Small-integer operands make gu exact, so gu must
    equal the plain product bitwise and a must equal the unfused swiglu_fwd of it; random operands are
    compared with the fp32 oracle of the same two steps."""
    torch.manual_seed(3)
    x = torch.randint(-2, 3, (M, d), device=gpu_device).to(torch.bfloat16)
    w = torch.randint(-1, 2, (2 * F, d), device=gpu_device).to(torch.bfloat16)
    gu, a = torch.ops.bpe_hip.gemm_swiglu_fwd(x, w)
    gu_ref = (x.float() @ w.float().t()).to(torch.bfloat16)
    assert torch.equal(gu, gu_ref)
    assert torch.equal(a, torch.ops.bpe_hip.swiglu_fwd(gu_ref))
    x = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    w = (0.1 * torch.randn(2 * F, d, device=gpu_device)).to(torch.bfloat16)
    gu, a = torch.ops.bpe_hip.gemm_swiglu_fwd(x, w)
    ref = x.float() @ w.float().t()
    assert rel(gu.cpu(), ref.cpu()) < 1e-2
    g, u = ref[:, :F], ref[:, F:]
    assert rel(a.cpu(), (g * torch.sigmoid(g) * u).cpu()) < 2e-2


@pytest.mark.parametrize("H,Hkv,D", [(8, 2, 64), (4, 4, 64), (4, 2, 128)])
def test_gemm_qkv_rope(gpu_device, gpp_mode, H, Hkv, D):
    """QKV projection with RoPE in the GEMM epilogue vs the unfused pair (matmul, then rope_qk_ in place).  Small
    integer operands make every product exact, so the two must agree bitwise (the RoPE arithmetic is the same
    fp32 formula on the same bf16 values); the partly rotated tile (Q / K end inside a 256-column tile) and the
    untouched V columns are both covered."""
    from bpe_transformer.ops import reference as R
    h = torch.ops.bpe_hip
    B, S, d = 2, 256, 256
    N = (H + 2 * Hkv) * D
    g = torch.Generator(device="cpu").manual_seed(H * 10 + Hkv)
    x = torch.randint(-2, 3, (B * S, d), generator=g).to(torch.bfloat16).to(gpu_device)
    w = torch.randint(-1, 2, (N, d), generator=g).to(torch.bfloat16).to(gpu_device)
    cos, sin = R.rope_tables(D, 1024, 10000.0, device=gpu_device)
    ref = torch.matmul(x, w.t())
    h.rope_qk_(ref, cos, sin, B, S, H, Hkv, D)
    out = h.gemm_qkv_rope(x, w, cos, sin, S, D, (H + Hkv) * D)
    assert torch.equal(out, ref)
    # random operands against the fp32 oracle (rotation of the bf16-rounded product)
    x = torch.randn(B * S, d, device=gpu_device, dtype=torch.bfloat16)
    w = (0.1 * torch.randn(N, d, device=gpu_device)).to(torch.bfloat16)
    out = h.gemm_qkv_rope(x, w, cos, sin, S, D, (H + Hkv) * D)
    y = (x.float() @ w.float().t()).to(torch.bfloat16)
    h.rope_qk_(y, cos, sin, B, S, H, Hkv, D)
    assert rel(out.float().cpu(), y.float().cpu()) < 1e-2


def test_gemm_pp_persistent_bitwise_many_tiles(gpu_device):
    """More tiles than CUs (every workgroup walks several, the last round partial): the persistent kernel runs the
    same per-tile MFMA sequence as the one-tile kernel, so plain, SwiGLU-forward and SwiGLU-backward outputs must
    match it bitwise."""
    h = torch.ops.bpe_hip
    torch.manual_seed(5)
    M, d, F = 8448, 768, 1024  # 33 x 9 = 297 plain tiles, 33 x 8 = 264 SwiGLU-forward, 33 x 4 = 132 backward
    x = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    w = (0.05 * torch.randn(2304, d, device=gpu_device)).to(torch.bfloat16)
    w13 = (0.05 * torch.randn(2 * F, d, device=gpu_device)).to(torch.bfloat16)
    w2 = (0.05 * torch.randn(d, F, device=gpu_device)).to(torch.bfloat16)
    dy = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    outs = {}
    prev = h.gpp_persist_config(0)
    try:
        for mode in (0, 1):
            h.gpp_persist_config(mode)
            c = torch.empty(M, 2304, device=gpu_device, dtype=torch.bfloat16)
            h.gemm_pp(x, True, w, True, c, 0.0, 1)
            gu, a = h.gemm_swiglu_fwd(x, w13)
            dgu = h.gemm_swiglu_bwd(dy, w2, gu)
            outs[mode] = (c, gu, a, dgu)
    finally:
        h.gpp_persist_config(prev)
    for t0, t1 in zip(outs[0], outs[1]):
        assert torch.equal(t0, t1)
    assert rel(outs[1][0].cpu(), (x.float() @ w.float().t()).cpu()) < 1e-2


@pytest.mark.parametrize("persist", [0, 1, 40])
def test_gemm_pp_tile_order_bitwise(gpu_device, persist):
    """Column-major tile bands (gpp_order_config gm > 0) only change which workgroup computes a tile: plain, QKV +
    RoPE, SwiGLU-forward and SwiGLU-backward outputs must equal the row-major ones bitwise, including the ragged
    last band (33 row blocks) and, at persist = 40, many tiles per workgroup."""
    h = torch.ops.bpe_hip
    torch.manual_seed(6)
    M, d, F, S, D = 8448, 768, 1024, 256, 64
    x = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    w = (0.05 * torch.randn(2304, d, device=gpu_device)).to(torch.bfloat16)
    w13 = (0.05 * torch.randn(2 * F, d, device=gpu_device)).to(torch.bfloat16)
    w2 = (0.05 * torch.randn(d, F, device=gpu_device)).to(torch.bfloat16)
    dy = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    ang = torch.arange(S, device=gpu_device, dtype=torch.float32)[:, None] * torch.rand(D // 2, device=gpu_device)
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    outs = {}
    prev_p, prev_o = h.gpp_persist_config(persist), h.gpp_order_config(-1)
    try:
        for gm in (0, 2, 4, 8, 16):
            h.gpp_order_config(gm)
            c = torch.empty(M, 2304, device=gpu_device, dtype=torch.bfloat16)
            h.gemm_pp(x, True, w, True, c, 0.0, 1)
            q = h.gemm_qkv_rope(x, w, cos, sin, S, D, 1536)
            gu, a = h.gemm_swiglu_fwd(x, w13)
            dgu = h.gemm_swiglu_bwd(dy, w2, gu)
            outs[gm] = (c, q, gu, a, dgu)
    finally:
        h.gpp_persist_config(prev_p)
        h.gpp_order_config(prev_o)
    for gm in (2, 4, 8, 16):
        for t0, t1 in zip(outs[0], outs[gm]):
            assert torch.equal(t0, t1), gm
    assert rel(outs[0][0].cpu(), (x.float() @ w.float().t()).cpu()) < 1e-2


@pytest.mark.parametrize("x_k", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_pp_dw_group_exact(gpu_device, x_k, dtype, splits):
    """Grouped weight gradients on small-integer operands: three problems of different shapes and strides (one a
    column slice of a wider buffer, like a stacked-weight gradient view) in one launch, every output exact."""
    torch.manual_seed(3)
    R = 1216
    shapes = [(512, 768), (256, 256), (768, 512)]
    gs, dys, xs, refs = [], [], [], []
    for i, (m, n) in enumerate(shapes):
        dy = torch.randint(-1, 2, (R, m), device=gpu_device).to(torch.bfloat16)
        x = torch.randint(-1, 2, (R, n), device=gpu_device).to(torch.bfloat16)
        wide = torch.randint(-3, 4, (m, n + 256 * i), device=gpu_device).to(dtype)
        g = wide[:, 256 * i :]  # a strided view: row stride != N for i > 0
        refs.append(g.float() + dy.float().t() @ x.float())
        gs.append(g)
        dys.append(dy)
        xs.append(x.t().contiguous() if x_k else x)
    torch.ops.bpe_hip.gemm_pp_dw_group(gs, dys, xs, x_k, splits, 1.0)
    for g, ref in zip(gs, refs):
        assert torch.equal(g.float().cpu(), ref.cpu())


def test_gemm_pp_dw_group_bitwise_vs_single(gpu_device, monkeypatch):
    """Random operands at GPT-2-like dW shapes (more workgroups than CUs): the grouped launch runs each tile's
    split exactly as the single-problem split-K kernel does and reduces in the same split order, so every
    gradient matches the per-shape ``gemm_pp`` route bitwise; repeated launches are bitwise stable."""
    from bpe_transformer.ops import gemm
    from bpe_transformer.ops.gemm import accumulate_weight_grads, choose_splits_group

    monkeypatch.setattr(gemm, "_GROUP", True)  # the grouped launch is opt-in (BPE_DW_GROUP=1)
    torch.manual_seed(4)
    T = 16384
    shapes = [(768, 2048), (4096, 768)]  # W2 and [W1; W3] of GPT-2-small: 24 + 48 tiles
    dys = [torch.randn(T, m, device=gpu_device, dtype=torch.bfloat16) * 0.1 for m, _ in shapes]
    xs = [torch.randn(T, n, device=gpu_device, dtype=torch.bfloat16) for _, n in shapes]
    g0 = [torch.randn(m, n, device=gpu_device, dtype=torch.bfloat16) for m, n in shapes]
    s = choose_splits_group(72, T, sum(m * n for m, n in shapes))
    single = [g.clone() for g in g0]
    for g, dy, x in zip(single, dys, xs):
        torch.ops.bpe_hip.gemm_pp(dy, False, x, False, g, 1.0, s)
    for _ in range(2):
        grouped = [g.clone() for g in g0]
        accumulate_weight_grads(list(zip(grouped, dys, xs)))
        for a, b in zip(grouped, single):
            assert torch.equal(a, b)
    ref = g0[1].float() + dys[1].float().t() @ xs[1].float()
    assert rel(grouped[1].cpu(), ref.cpu()) < 1e-2


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_pp_exact(gpu_device, gpp_mode, a_k, b_k, splits):
    """Ping-pong GEMM on small-integer operands: every output is exact, so any layout/index slip shows."""
    torch.manual_seed(1)
    M, N, R = 512, 768, 448
    A = torch.randint(-1, 2, (M, R), device=gpu_device).to(torch.bfloat16)
    B = torch.randint(-1, 2, (N, R), device=gpu_device).to(torch.bfloat16)
    Am = A if a_k else A.t().contiguous()
    Bm = B if b_k else B.t().contiguous()
    C = torch.randint(-3, 4, (M, N), device=gpu_device).to(torch.bfloat16)
    ref = C.float() * 2.0 + A.float() @ B.float().t()
    torch.ops.bpe_hip.gemm_pp(Am, a_k, Bm, b_k, C, 2.0, splits)
    assert torch.equal(C.float().cpu(), ref.cpu())


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False)])
def test_gemm_pp_random(gpu_device, gpp_mode, a_k, b_k):
    torch.manual_seed(0)
    M, N, R = 1024, 512, 1536
    A = torch.randn(M, R, device=gpu_device, dtype=torch.bfloat16)
    B = torch.randn(N, R, device=gpu_device, dtype=torch.bfloat16)
    Am = A if a_k else A.t().contiguous()
    Bm = B if b_k else B.t().contiguous()
    C = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
    torch.ops.bpe_hip.gemm_pp(Am, a_k, Bm, b_k, C, 0.0, 1 if a_k else 4)
    ref = A.float() @ B.float().t()
    assert rel(C.cpu(), ref.cpu()) < 1e-2


@pytest.mark.parametrize("shape", [(2304, 768, 8192), (768, 768, 8192), (11264, 2048, 2048), (2048, 5632, 4096),
                                   (50432, 256, 4096), (768, 768, 65536)])
def test_weight_grad_shapes(gpu_device, shape):
    """Model dW shapes through the routing in ops.gemm (256-tile kernel, split-K choice)."""
    from bpe_transformer.ops.gemm import accumulate_weight_grad

    n, k, t = shape
    torch.manual_seed(0)
    dy = torch.randn(t, n, device=gpu_device, dtype=torch.bfloat16)
    x = torch.randn(t, k, device=gpu_device, dtype=torch.bfloat16)
    g = torch.randn(n, k, device=gpu_device, dtype=torch.bfloat16)
    ref = g.float() + dy.float().t() @ x.float()
    accumulate_weight_grad(g, dy, x)
    assert rel(g, ref) < 1e-2


@pytest.mark.parametrize("route", ["pp", "ppt", "hip256"])
@pytest.mark.parametrize("shape", [(2304, 768, 8192), (1024, 2048, 4096)])
def test_weight_grad_routes(gpu_device, route, shape):
    """Each dW route of ops.gemm on its own (ppt: the ping-pong kernel on a transposed copy of X), accumulating into
    g, against the fp32 product."""
    from bpe_transformer.ops.gemm import _run

    n, k, t = shape
    torch.manual_seed(1)
    dy = torch.randn(t, n, device=gpu_device, dtype=torch.bfloat16)
    x = torch.randn(t, k, device=gpu_device, dtype=torch.bfloat16)
    g = torch.randn(n, k, device=gpu_device, dtype=torch.bfloat16)
    ref = g.float() + dy.float().t() @ x.float()
    _run(route, g, dy, x)
    assert rel(g, ref) < 1e-2


def test_weight_grad_accumulate(gpu_device):
    from bpe_transformer.ops.gemm import accumulate_weight_grad

    torch.manual_seed(0)
    dy = torch.randn(4096, 768, device=gpu_device, dtype=torch.bfloat16)
    x = torch.randn(4096, 2304, device=gpu_device, dtype=torch.bfloat16)
    g = torch.randn(768, 2304, device=gpu_device, dtype=torch.bfloat16)
    ref = g.float() + dy.float().t() @ x.float()
    accumulate_weight_grad(g, dy, x)
    assert rel(g.cpu(), ref.cpu()) < 1e-2


# ---------------------------------------------------------------- flash attention
def _fa_case(gpu_device, B, S, H, Hkv, D, rope, causal, seed=0, prerotate=None):
    torch.manual_seed(seed)
    W = (H + 2 * Hkv) * D
    qkv = torch.randn(B * S, W, device=gpu_device, dtype=torch.bfloat16).requires_grad_(True)
    cos = sin = None
    if rope:
        cos, sin = R.rope_tables(D, S + 16, 10000.0, device=gpu_device)
    o = ops.flash_attention_qkv(qkv, B, S, H, Hkv, D, cos, sin, causal, prerotate=prerotate)
    do = torch.randn_like(o)
    o.backward(do)
    qr = qkv.detach().float().cpu().requires_grad_(True)
    orf = ops.attention_qkv_reference(qr, B, S, H, Hkv, D, None if cos is None else cos.cpu(),
                                      None if sin is None else sin.cpu(), causal)
    orf.backward(do.float().cpu())
    return o, qkv.grad, orf.detach(), qr.grad


@pytest.mark.parametrize("S", [128, 256, 200, 64, 1000])
@pytest.mark.parametrize("rope", ["fused", "prerotated", None])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_d64(gpu_device, S, rope, causal):
    """D = 64: fused-RoPE kernels (rope "fused"), the v3 forward with Q / K rotated by rope_qk_ ("prerotated")
    and without RoPE (None, v3 forward); S not a multiple of 64 covers the clamped DMA rows and masked tail."""
    o, g, orf, gr = _fa_case(gpu_device, 2, S, 4, 4, 64, rope is not None, causal, prerotate=rope == "prerotated")
    assert rel(o.cpu(), orf) < 2e-2, rel(o.cpu(), orf)
    HD = 4 * 64
    for name, sl in (("dq", slice(0, HD)), ("dk", slice(HD, 2 * HD)), ("dv", slice(2 * HD, 3 * HD))):
        e = rel(g[:, sl].cpu(), gr[:, sl])
        assert e < 3e-2, (name, e)


@pytest.mark.parametrize("pre", [True, False])
@pytest.mark.parametrize("D,H,Hkv", [(128, 4, 4), (64, 8, 2), (128, 8, 4), (64, 32, 4)])
def test_flash_attention_d128_and_gqa(gpu_device, D, H, Hkv, pre):
    o, g, orf, gr = _fa_case(gpu_device, 2, 192, H, Hkv, D, True, True, seed=1, prerotate=pre)
    assert rel(o.cpu(), orf) < 2e-2
    assert rel(g.cpu(), gr) < 3e-2


def test_flash_attention_gpt2_shape(gpu_device):
    o, g, orf, gr = _fa_case(gpu_device, 1, 1024, 12, 12, 64, True, True, seed=2)
    assert rel(o.cpu(), orf) < 2e-2
    assert rel(g.cpu(), gr) < 3e-2


@pytest.mark.parametrize("S", [1024, 200, 64])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_fwd_versions_agree(gpu_device, S, causal):
    """The D = 64 forward on pre-rotated Q / K (v8, flash_attn_fwd_v4.hip: LDS-DMA K / V, no tile max on the common
    path) against the general kernel (v2, fa_fwd_kernel) -- O within bf16 rounding, LSE within 1e-2 (log2 units)."""
    h = torch.ops.bpe_hip
    B, H, D = 2, 4, 64
    torch.manual_seed(5)
    x = torch.randn(B * S, 3 * H * D, device=gpu_device, dtype=torch.bfloat16)
    q, k, v = x[:, : H * D], x[:, H * D : 2 * H * D], x[:, 2 * H * D :]
    e = torch.empty(0, 0, device=gpu_device)
    prev = h.fa_fwd_config(2)
    try:
        o2, l2 = h.fa_fwd(q, k, v, e, e, B, S, H, H, D, causal, False, D ** -0.5, False)
        h.fa_fwd_config(8)
        o8, l8 = h.fa_fwd(q, k, v, e, e, B, S, H, H, D, causal, False, D ** -0.5, False)
    finally:
        h.fa_fwd_config(prev)
    assert prev == 8, "the default D = 64 forward is v8"
    assert rel(o8.float().cpu(), o2.float().cpu()) < 1e-2
    assert (l8 - l2).abs().max().item() < 1e-2


@pytest.fixture
def fused_bwd():
    """Run the test with the fused (fp32-atomics) attention backward, the one that owns the dQ accumulator and the
    pre-pass / convert kernels (D = 64 defaults to the split form, csrc/flash_attn_bwd_split.hip)."""
    h = torch.ops.bpe_hip
    prev = h.fa_bwd_config(1)  # returns the form in force before the call
    yield
    h.fa_bwd_config(prev)
    assert h.fa_bwd_config(-1) == 0, "the default D = 64 backward is the split form"


@pytest.mark.parametrize("S", [1024, 200, 64, 1000])
@pytest.mark.parametrize("H,Hkv", [(4, 4), (8, 2)])
@pytest.mark.parametrize("rope", ["fused", "prerotated", None])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_bwd_split_vs_fused_and_oracle(gpu_device, S, H, Hkv, rope, causal):
    """The split backward (dQ kernel + dK/dV kernel: LDS-DMA 128-row tiles, or register-staged 64-row tiles with
    RoPE fused, rope == "fused") against the fp32 oracle's autograd and against the fused atomics backward on the
    same forward outputs: dQ, dK, dV each; and bitwise deterministic."""
    _split_vs_fused(gpu_device, S, H, Hkv, 64, rope, causal)


@pytest.mark.parametrize("S", [1024, 200, 64])
@pytest.mark.parametrize("H,Hkv", [(4, 4), (8, 2)])
@pytest.mark.parametrize("rope", ["fused", "prerotated", None])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_bwd_split_d128(gpu_device, S, H, Hkv, rope, causal):
    """The split backward at D = 128 (256-byte rows, 64-row LDS-DMA tiles; rope "fused": fa_bwd rotates a copy of Q /
    K and runs the pre-rotated kernels) against the oracle and the fused atomics form, and bitwise deterministic."""
    _split_vs_fused(gpu_device, S, H, Hkv, 128, rope, causal)


def _split_vs_fused(gpu_device, S, H, Hkv, D, rope, causal):
    h = torch.ops.bpe_hip
    B = 2
    torch.manual_seed(11)
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device=gpu_device, dtype=torch.bfloat16)
    use_rope = rope is not None
    cos, sin = R.rope_tables(D, S + 5, 10000.0, device=gpu_device)
    pre = rope == "prerotated"
    x = qkv.clone()
    if pre:
        h.rope_qk_(x, cos, sin, B, S, H, Hkv, D)
    q, k, v = x[:, : H * D], x[:, H * D : (H + Hkv) * D], x[:, (H + Hkv) * D :]
    scale = D ** -0.5
    o, lse = h.fa_fwd(q, k, v, cos, sin, B, S, H, Hkv, D, causal, use_rope, scale, pre)
    do = torch.randn_like(o)
    assert h.fa_bwd_config(-1) == 0, "the default backward is the split form"
    assert not h.fa_bwd_needs_dq_acc(D), "the split form takes no fp32 dQ accumulator"
    try:
        got = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, use_rope, scale, pre)
        again = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, use_rope, scale, pre)
        h.fa_bwd_config(1)
        fused = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, use_rope, scale, pre)
    finally:
        h.fa_bwd_config(0)
    assert torch.equal(got, again), "split backward is not deterministic"
    qr = qkv.float().cpu().requires_grad_(True)
    orf = ops.attention_qkv_reference(qr, B, S, H, Hkv, D, cos.cpu() if use_rope else None,
                                      sin.cpu() if use_rope else None, causal)
    orf.backward(do.float().cpu())
    gr = qr.grad
    HD, KD = H * D, Hkv * D
    for name, sl in (("dq", slice(0, HD)), ("dk", slice(HD, HD + KD)), ("dv", slice(HD + KD, HD + 2 * KD))):
        e = rel(got[:, sl].float().cpu(), gr[:, sl])
        ef = rel(fused[:, sl].float().cpu(), gr[:, sl])
        # the split kernels fold the softmax scale into bf16 Q (dQ kernel, as the forward does) / K (dK/dV kernel):
        # one more bf16 rounding in the recomputed scores than the fused kernel's fp32 scaling
        assert e < 3e-2 and e < 2.0 * ef + 2e-3, (name, e, ef)


@pytest.mark.parametrize("S", [1024, 200, 64, 1000, 136])
@pytest.mark.parametrize("H,Hkv", [(4, 4), (8, 2)])
@pytest.mark.parametrize("pre", [True, False])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("form", [1, 2], ids=["nw8_kt128", "nw4_kt64"])
def test_flash_bwd_dq16_vs_dq32_and_oracle(gpu_device, S, H, Hkv, pre, causal, form):
    """The split backward's dQ kernel with 16 queries per wave (flash_attn_bwd_dq16.hip: 16x16x32 MFMAs, 4 waves per
    SIMD, its own LDS swizzle; form 1: 8 waves and 128-key tiles, form 2: 4 waves and 64-key tiles) against the 32-query kernel and the fp32 oracle's autograd: dQ within the oracle
    bound and no worse than the 32-row kernel's error; dV bitwise equal (no delta in it); dK within fp32 rounding
    of delta's summation order; bitwise repeatable.  S 136 and 1000 cover partial query blocks and key tiles."""
    h = torch.ops.bpe_hip
    B, D = 2, 64
    torch.manual_seed(17)
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device=gpu_device, dtype=torch.bfloat16)
    cos, sin = R.rope_tables(D, S + 5, 10000.0, device=gpu_device)
    x = qkv.clone()
    if pre:
        h.rope_qk_(x, cos, sin, B, S, H, Hkv, D)
    q, k, v = x[:, : H * D], x[:, H * D : (H + Hkv) * D], x[:, (H + Hkv) * D :]
    scale = D ** -0.5
    o, lse = h.fa_fwd(q, k, v, cos, sin, B, S, H, Hkv, D, causal, pre, scale, pre)
    do = torch.randn_like(o)
    prev = h.fa_dq_config(form)
    try:
        g16 = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, pre, scale, pre)
        again = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, pre, scale, pre)
        h.fa_dq_config(0)
        g32 = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, pre, scale, pre)
    finally:
        h.fa_dq_config(prev)
    assert prev == 3, "the default dQ form: the 16-row kernel (8 waves) up to S = 2048, the 32-row one above"
    assert torch.equal(g16, again), "dq16 backward is not deterministic"
    HD, KD = H * D, Hkv * D
    assert torch.equal(g16[:, HD + KD :], g32[:, HD + KD :]), "dV differs between the dQ forms"
    assert rel(g16[:, HD : HD + KD].float().cpu(), g32[:, HD : HD + KD].float().cpu()) < 2e-3
    qr = qkv.float().cpu().requires_grad_(True)
    orf = ops.attention_qkv_reference(qr, B, S, H, Hkv, D, cos.cpu() if pre else None, sin.cpu() if pre else None,
                                      causal)
    orf.backward(do.float().cpu())
    e16 = rel(g16[:, :HD].float().cpu(), qr.grad[:, :HD])
    e32 = rel(g32[:, :HD].float().cpu(), qr.grad[:, :HD])
    assert e16 < 3e-2 and e16 < 1.2 * e32 + 2e-3, (e16, e32)


@pytest.mark.parametrize("S,H,Hkv", [(1024, 8, 2), (200, 32, 4), (1000, 4, 1)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_bwd_gqa_head_sweep(gpu_device, S, H, Hkv, causal):
    """GQA dK / dV of the split backward: one workgroup per KV head sweeping its G query heads (no fp32 partials, no
    reduce kernel) against the fused backward's per-query-head partials + reduce form and against the fp32 oracle."""
    h = torch.ops.bpe_hip
    B, D = 2, 64
    torch.manual_seed(13)
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device=gpu_device, dtype=torch.bfloat16)
    cos, sin = R.rope_tables(D, S, 10000.0, device=gpu_device)
    x = qkv.clone()
    h.rope_qk_(x, cos, sin, B, S, H, Hkv, D)
    q, k, v = x[:, : H * D], x[:, H * D : (H + Hkv) * D], x[:, (H + Hkv) * D :]
    scale = D ** -0.5
    o, lse = h.fa_fwd(q, k, v, cos, sin, B, S, H, Hkv, D, causal, True, scale, True)
    do = torch.randn_like(o)
    try:
        sweep = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, True, scale, True)
        h.fa_bwd_config(1)
        part = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, causal, True, scale, True)
    finally:
        h.fa_bwd_config(0)
    qr = qkv.float().cpu().requires_grad_(True)
    orf = ops.attention_qkv_reference(qr, B, S, H, Hkv, D, cos.cpu(), sin.cpu(), causal)
    orf.backward(do.float().cpu())
    HD, KD = H * D, Hkv * D
    for name, sl in (("dq", slice(0, HD)), ("dk", slice(HD, HD + KD)), ("dv", slice(HD + KD, HD + 2 * KD))):
        es = rel(sweep[:, sl].float().cpu(), qr.grad[:, sl])
        ep = rel(part[:, sl].float().cpu(), qr.grad[:, sl])
        assert es < 3e-2 and es < 2.0 * ep + 2e-3, (name, es, ep)


@pytest.mark.parametrize("S,D,H,Hkv,fused", [(1000, 64, 4, 4, False), (192, 128, 8, 4, True), (64, 64, 4, 2, True),
                                              (320, 64, 4, 4, True)])
def test_flash_dq_acc_zeroed_by_forward(gpu_device, S, D, H, Hkv, fused, fused_bwd):
    """fa_fwd handed the backward's fp32 dQ accumulator (filled with NaN here) zeroes every row of it,
    padding included, and fa_bwd then skips its own zeroing: the gradients equal those of the path where the
    backward pre-pass zeroes (the fused blocks use this form) -- dK / dV bitwise, dQ up to the order of its fp32
    atomics."""
    torch.manual_seed(5)
    B = 2
    h = torch.ops.bpe_hip
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device=gpu_device, dtype=torch.bfloat16)
    cos, sin = R.rope_tables(D, S + 3, 10000.0, device=gpu_device)
    q, k, v = qkv[:, : H * D], qkv[:, H * D : (H + Hkv) * D], qkv[:, (H + Hkv) * D :]
    scale = D ** -0.5
    acc = torch.full((B * ((S + 63) // 64 * 64), H * D), float("nan"), device=gpu_device)
    o, lse = h.fa_fwd(q, k, v, cos, sin, B, S, H, Hkv, D, True, True, scale, not fused, acc)
    assert bool((acc == 0).all()), "forward left rows of the dQ accumulator unzeroed"
    o2, lse2 = h.fa_fwd(q, k, v, cos, sin, B, S, H, Hkv, D, True, True, scale, not fused)
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    do = torch.randn_like(o)
    ref = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, True, True, scale, not fused)
    got = h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, True, True, scale, not fused, acc)
    assert torch.equal(got[:, H * D :], ref[:, H * D :])  # dK / dV: no atomics, bitwise
    assert rel(got[:, : H * D].cpu(), ref[:, : H * D].float().cpu()) < 1e-3  # dQ: fp32 atomics, order varies


def test_flash_bwd_streaming_path_matches(gpu_device, fused_bwd):
    """Past 128 MB of bf16 activation the backward's pre-pass / dQ-convert kernels switch to non-temporal loads
    (csrc/flash_attn_bwd.hip big_stream).  Batch 96 at the GPT-2 shape takes that path; its gradients must
    equal those of two 48-sequence halves, which take the plain path: dK / dV bitwise, dQ up to atomic order."""
    torch.manual_seed(6)
    B, S, H, D = 96, 1024, 12, 64
    assert B * S * H * D * 2 > (128 << 20) and B // 2 * S * H * D * 2 <= (128 << 20)
    h = torch.ops.bpe_hip
    qkv = torch.randn(B * S, 3 * H * D, device=gpu_device, dtype=torch.bfloat16)
    cos, sin = R.rope_tables(D, S, 10000.0, device=gpu_device)
    scale = D ** -0.5

    def run(x, b):
        q, k, v = x[:, : H * D], x[:, H * D : 2 * H * D], x[:, 2 * H * D :]
        o, lse = h.fa_fwd(q, k, v, cos, sin, b, S, H, H, D, True, True, scale, True)
        do = torch.ones_like(o) * 0.01 + (o * 0.5)
        return h.fa_bwd(do, q, k, v, o, lse, cos, sin, b, S, H, H, D, True, True, scale, True)

    full = run(qkv, B)
    half = torch.cat([run(qkv[: B // 2 * S], B // 2), run(qkv[B // 2 * S :], B // 2)])
    assert torch.equal(full[:, H * D :], half[:, H * D :])
    assert rel(full[:, : H * D], half[:, : H * D]) < 1e-3


@pytest.mark.parametrize("H,Hkv,D", [(4, 2, 64), (32, 4, 64), (12, 12, 64), (4, 4, 128)])
def test_rope_qk_inplace(gpu_device, H, Hkv, D):
    """rope_qk_ rotates exactly the Q and K heads of the fused activation (positions restart per sequence); chunk
    columns per row 48 / 288 / 192 / 128 cover partial and whole 64-column blocks, 200 rows a partial row group."""
    torch.manual_seed(4)
    B, S = 2, 100
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device=gpu_device, dtype=torch.bfloat16)
    cos, sin = R.rope_tables(D, S + 7, 10000.0, device=gpu_device)
    out = qkv.clone()
    torch.ops.bpe_hip.rope_qk_(out, cos, sin, B, S, H, Hkv, D)
    x = qkv.float().cpu().view(B, S, H + 2 * Hkv, D).transpose(1, 2)  # [B, heads, S, D]
    ref = x.clone()
    ref[:, : H + Hkv] = R.apply_rope(x[:, : H + Hkv], cos.cpu(), sin.cpu())
    ref = ref.transpose(1, 2).reshape(B * S, -1)
    assert rel(out.float().cpu(), ref) < 1e-2
    assert torch.equal(out[:, (H + Hkv) * D :], qkv[:, (H + Hkv) * D :])  # V untouched


def test_flash_attention_large_scores(gpu_device):
    """Spike one key so the running max jumps mid-sequence (forces the online-softmax rescale)."""
    torch.manual_seed(3)
    B, S, H, D = 1, 256, 2, 64
    qkv = torch.randn(B * S, 3 * H * D, device=gpu_device, dtype=torch.bfloat16)
    qkv[100, H * D : 2 * H * D] *= 8  # key row 100 large
    qkv[:, : H * D] *= 3
    qkv.requires_grad_(True)
    o = ops.flash_attention_qkv(qkv, B, S, H, H, D, None, None, True)
    orf = ops.attention_qkv_reference(qkv.detach().float().cpu(), B, S, H, H, D, None, None, True)
    assert rel(o.detach().cpu(), orf) < 2e-2


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [4096, 1000003, 37])
def test_cast_fp8_and_amax(gpu_device, dtype, n, fmt):
    """Saturating e4m3fn / e5m2 cast (incl. values beyond the range after scaling) + amax recording."""
    torch.manual_seed(0)
    fdt, fmax, big = ((torch.float8_e4m3fn, 448.0, 300.0) if fmt == "e4m3" else (torch.float8_e5m2, 57344.0, 30000.0))
    x = (torch.randn(n, device=gpu_device) * 3).to(dtype)
    x[n // 2] = big  # saturates at scale 4
    scale = torch.tensor([4.0], device=gpu_device)
    out = torch.empty(n, dtype=fdt, device=gpu_device)
    amax = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    torch.ops.bpe_hip.cast_fp8(x.contiguous(), scale, out, amax)
    ref = (x.float() * 4.0).clamp(-fmax, fmax).to(fdt)
    assert torch.equal(out.view(torch.uint8), ref.view(torch.uint8))
    assert amax.view(torch.float32).item() == x.float().abs().max().item()


# (192, 320): the 64 x 64 kernel; the others the 128 x 128 one, (8192, 4224) with more tiles than the grid (2112 >
# 2048: stride loop)
@pytest.mark.parametrize("N,K", [(192, 320), (4096, 1024), (384, 256), (8192, 4096), (8192, 4224)])
@pytest.mark.parametrize("fmt", [torch.float8_e4m3fn, torch.float8_e5m2])
def test_cast_fp8_transposed(gpu_device, N, K, fmt):
    """Two-layout cast (weights; activations and gradients of the fp8 weight-gradient GEMM): both layouts from one
    pass, identical bytes to the plain cast of the same format, amax folded in."""
    torch.manual_seed(3)
    w = torch.randn(N, K, device=gpu_device, dtype=torch.bfloat16) * 3
    scale = torch.tensor([4.0], device=gpu_device)
    amax = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    w8 = torch.empty(N, K, dtype=fmt, device=gpu_device)
    w8t = torch.empty(K, N, dtype=fmt, device=gpu_device)
    torch.ops.bpe_hip.cast_fp8_t(w, scale, w8, w8t, amax)
    ref = torch.empty_like(w8)
    torch.ops.bpe_hip.cast_fp8(w, scale, ref, torch.zeros(1, dtype=torch.int32, device=gpu_device))
    assert torch.equal(w8.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(w8t.view(torch.uint8), ref.view(torch.uint8).t().contiguous())
    am = amax.view(torch.float32).item()
    assert am == float(w.float().abs().max())


# (256, 192): the 64 x 64 kernel; (32768, 1408): 2816 tiles of 128 x 128, more than the grid (stride loop)
@pytest.mark.parametrize("M,F", [(256, 192), (1024, 512), (32768, 1408)])
def test_swiglu_cast_fp8_transposed(gpu_device, M, F):
    """SwiGLU with the two-layout fp8 cast fused (fp8.hip swiglu_cast_fp8_t): forward a = silu(g) u as e4m3 [M, F] and
    [F, M], backward [dg | du] as e5m2 [M, 2F] and [2F, M] -- against the two-pass form (swiglu_fwd / swiglu_bwd to
    bf16, then cast_fp8_t) on the same scale: the kernels round to bf16 first, so the bytes and the amax agree (up to
    the rare value whose bf16 rounding the compiler's fused multiply-adds move by one ulp)."""
    from bpe_transformer.ops.fp8 import Fp8State, swiglu_bwd_cast_t, swiglu_fwd_cast_t
    h = torch.ops.bpe_hip
    torch.manual_seed(7)
    gu = torch.randn(M, 2 * F, device=gpu_device, dtype=torch.bfloat16) * 2
    da = torch.randn(M, F, device=gpu_device, dtype=torch.bfloat16) * 0.01

    def two_pass(x, fmt, scale):
        amax = torch.zeros(1, dtype=torch.int32, device=gpu_device)
        x8 = torch.empty(x.shape, dtype=fmt, device=gpu_device)
        x8t = torch.empty(x.shape[1], x.shape[0], dtype=fmt, device=gpu_device)
        h.cast_fp8_t(x, scale, x8, x8t, amax)
        return x8, x8t, amax.view(torch.float32).item()

    for fwd in (True, False):
        st = Fp8State(1, gpu_device, fmt="e4m3" if fwd else "e5m2")
        st.scale.fill_(8.0 if fwd else 2048.0)
        if fwd:
            o8, o8t = swiglu_fwd_cast_t(st, gu, 0)
            r8, r8t, ram = two_pass(h.swiglu_fwd(gu), st.dtype, st.scale[:1])
        else:
            o8, o8t = swiglu_bwd_cast_t(st, da, gu, 0)
            r8, r8t, ram = two_pass(h.swiglu_bwd(da, gu), st.dtype, st.scale[:1])
        assert torch.equal(o8t.view(torch.uint8), o8.view(torch.uint8).t().contiguous())
        diff = (o8.view(torch.uint8) != r8.view(torch.uint8)).float().mean().item()
        assert diff < 1e-3, (fwd, diff)
        assert rel(o8.float(), r8.float()) < 1e-2
        am = st.amax.view(torch.float32).item()
        assert abs(am - ram) <= 1e-2 * ram, (fwd, am, ram)


@pytest.mark.parametrize("M,N,add", [(256, 256, True), (1024, 2048, True), (384, 768, False)])
def test_add_rmsnorm_cast_fp8_transposed(gpu_device, M, N, add):
    """Residual add + RMSNorm written only as e4m3 in both layouts (fp8.hip add_rmsnorm_fp8_kernel + the fp8
    transpose) against add_rmsnorm_fwd / rmsnorm_fwd followed by the two-layout cast: same sum and rstd, fp8 bytes
    equal up to rare one-ulp bf16 differences, same amax."""
    from bpe_transformer.ops.fp8 import Fp8State, add_rmsnorm_cast_t
    h = torch.ops.bpe_hip
    torch.manual_seed(9)
    x = torch.randn(M, N, device=gpu_device, dtype=torch.bfloat16)
    d = torch.randn(M, N, device=gpu_device, dtype=torch.bfloat16) if add else None
    w = (1 + 0.1 * torch.randn(N, device=gpu_device)).to(torch.bfloat16)
    st = Fp8State(1, gpu_device)
    st.scale.fill_(16.0)
    s, (y8, y8t), rstd = add_rmsnorm_cast_t(st, x, d, w, 1e-5, 0)
    if add:
        s_ref, y_ref, r_ref = h.add_rmsnorm_fwd(x, d, w, 1e-5)
        assert torch.equal(s, s_ref)
    else:
        y_ref, r_ref = h.rmsnorm_fwd(x, w, 1e-5)
        assert s is x
    assert rel(rstd, r_ref) < 1e-5
    amax = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    r8 = torch.empty(M, N, dtype=torch.float8_e4m3fn, device=gpu_device)
    r8t = torch.empty(N, M, dtype=torch.float8_e4m3fn, device=gpu_device)
    h.cast_fp8_t(y_ref, st.scale[:1], r8, r8t, amax)
    assert torch.equal(y8t.view(torch.uint8), y8.view(torch.uint8).t().contiguous())
    diff = (y8.view(torch.uint8) != r8.view(torch.uint8)).float().mean().item()
    assert diff < 1e-3, diff
    am, ram = st.amax.view(torch.float32).item(), amax.view(torch.float32).item()
    assert abs(am - ram) <= 1e-2 * ram, (am, ram)


@pytest.mark.parametrize("H,Hkv,D", [(8, 2, 64), (4, 2, 128)])
def test_gemm_fp8_rope(gpu_device, gpp_mode, H, Hkv, D):
    """The fp8 QKV projection with RoPE in the hand kernel's epilogue equals the same kernel without it followed by
    rope_qk_ in place (same bf16-rounded scaled products, same rotation arithmetic): bitwise."""
    from bpe_transformer.ops import reference as R
    h = torch.ops.bpe_hip
    torch.manual_seed(4)
    B, S, d = 2, 256, 256
    N = (H + 2 * Hkv) * D
    x8 = (torch.randn(B * S, d, device=gpu_device) * 4).to(torch.float8_e4m3fn)
    w8 = (torch.randn(N, d, device=gpu_device) * 4).to(torch.float8_e4m3fn)
    sa = torch.tensor([0.25], device=gpu_device)
    sb = torch.tensor([0.125], device=gpu_device)
    cos, sin = R.rope_tables(D, 1024, 10000.0, device=gpu_device)
    ref = h.gemm_fp8(x8, w8, sa, sb)
    h.rope_qk_(ref, cos, sin, B, S, H, Hkv, D)
    out = h.gemm_fp8_rope(x8, w8, sa, sb, cos, sin, S, D, (H + Hkv) * D)
    assert torch.equal(out, ref)


def test_fp8_grads_weight_gradient(gpu_device):
    """ops.fp8.grads: one e5m2 cast of the output gradient serves dX = g W and dW = g^T X; both against the fp32
    products of the dequantised operands (the weight-gradient GEMM reduces over all tokens: M = N_out, K = T)."""
    from bpe_transformer.ops.fp8 import Fp8State, grads
    torch.manual_seed(11)
    T, N, K = 8192, 512, 256
    xs = Fp8State(2, gpu_device)
    gs = Fp8State(1, gpu_device, fmt="e5m2")
    x = torch.randn(T, K, device=gpu_device, dtype=torch.bfloat16)
    w = (0.1 * torch.randn(N, K, device=gpu_device)).to(torch.bfloat16)
    g = (1e-3 * torch.randn(T, N, device=gpu_device)).to(torch.bfloat16)
    for _ in range(2):  # calibrate the delayed scales on the same tensors
        y, w8t, xt8 = xs.matmul(x, w, 0, 1, keep_w8=True, keep_xt=True)
        dx, dw = grads(gs, g, 0, w8t, xs, 1, xt8, xs, 0)
        xs.update()
        gs.update()
    y, w8t, xt8 = xs.matmul(x, w, 0, 1, keep_w8=True, keep_xt=True)
    dx, dw = grads(gs, g, 0, w8t, xs, 1, xt8, xs, 0)
    assert dx.shape == (T, K) and dw.shape == (N, K) and xt8.shape == (K, T)
    xq = xt8.float().t() * xs.inv_scale[0]
    g8 = gs.cast(g, 0).float() * gs.inv_scale[0]
    wq = w8t.float().t() * xs.inv_scale[1]
    assert rel(dw.float(), g8.t() @ xq) < 1e-2
    assert rel(dx.float(), g8 @ wq) < 1e-2
    assert rel(dw.float(), g.float().t() @ x.float()) < 0.1  # fp8 rounding of both operands


@pytest.mark.parametrize("c_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_fp8_acc_splitk(gpu_device, c_dtype, splits):
    """Split-K fp8 GEMM accumulating into C (the fp8 weight-gradient form): exact on small-integer operands with
    power-of-two scales, e5m2 x e4m3, beta = 1 onto an existing C."""
    g = torch.Generator(device="cpu").manual_seed(splits)
    M, N, K = 512, 256, 1536
    a = torch.randint(-4, 5, (M, K), generator=g).float()
    b = torch.randint(-4, 5, (N, K), generator=g).float()
    c0 = torch.randint(-8, 9, (M, N), generator=g).float()
    a8 = a.to(torch.float8_e5m2).to(gpu_device)
    b8 = b.to(torch.float8_e4m3fn).to(gpu_device)
    c = c0.to(c_dtype).to(gpu_device)
    sa = torch.tensor([0.5], device=gpu_device)
    sb = torch.tensor([0.25], device=gpu_device)
    torch.ops.bpe_hip.gemm_fp8_acc(a8, b8, sa, sb, c, 1.0, splits)
    ref = (c0 + (a @ b.t()) * 0.125).to(c_dtype)
    assert torch.equal(c.cpu(), ref)


def test_update_scales(gpu_device):
    n, H = 3, 4
    amax = torch.tensor([2.0, 0.0, 1000.0], device=gpu_device).view(torch.int32).clone()
    hist = torch.zeros(n, H, device=gpu_device)
    hist[2, 1] = 3000.0  # older, larger amax dominates the window
    scale = torch.ones(n, device=gpu_device)
    inv = torch.ones(n, device=gpu_device)
    torch.ops.bpe_hip.update_scales(amax, hist, scale, inv, 0, 1.0, 0)
    assert scale.tolist() == [128.0, 1.0, 0.125]  # 2^floor(log2(448 / amax))
    assert torch.allclose(inv * scale, torch.ones(n, device=gpu_device))
    assert amax.tolist() == [0, 0, 0]
    assert hist[:, 0].tolist() == [2.0, 0.0, 1000.0]
    # e5m2 (gradients): 2^floor(log2(57344 / amax))
    amax.copy_(torch.tensor([2.0, 0.0, 1000.0], device=gpu_device).view(torch.int32))
    torch.ops.bpe_hip.update_scales(amax, hist, scale, inv, 1, 1.0, 1)
    assert scale.tolist() == [16384.0, 1.0, 32.0]  # row 2: pos 1 overwrote the old 3000 -> max 1000


# ---------------------------------------------------------------- hand-written fp8 GEMM (gemm_pp.hip, F8)
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 256, 384), (256, 768, 1024)])
@pytest.mark.parametrize("fmt_a", ["e4m3", "e5m2"])
def test_gemm_fp8_exact(gpu_device, gpp_mode, M, N, K, fmt_a):
    """y = (a8 @ b8^T) * sa * sb on the fp8 MFMA ping-pong kernel, exact on small-integer operands (fp32 sums of
    integers are exact; the bf16 output is the round-to-nearest of the exact value) with power-of-two scales:
    checks the fragment / k mapping of v_mfma_scale_f32_16x16x128_f8f6f4 for both operand formats."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randint(-4, 5, (M, K), generator=g).float()
    b = torch.randint(-4, 5, (N, K), generator=g).float()
    a[3, :] = 0.0  # an all-zero row and column
    b[:, 5] = 0.0
    dt_a = torch.float8_e4m3fn if fmt_a == "e4m3" else torch.float8_e5m2
    a8 = a.to(dt_a).to(gpu_device)
    b8 = b.to(torch.float8_e4m3fn).to(gpu_device)
    sa = torch.tensor([0.25], device=gpu_device)
    sb = torch.tensor([2.0], device=gpu_device)
    y = torch.ops.bpe_hip.gemm_fp8(a8, b8, sa, sb)
    ref = ((a @ b.t()) * 0.5).to(torch.bfloat16)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    assert torch.equal(y.cpu(), ref)


@pytest.mark.parametrize("M,F,K,persist", [(512, 384, 256, 1), (4096, 640, 512, 40), (1024, 5632, 2048, 1)])
def test_gemm_fp8_swiglu_matches_gemm_then_cast(gpu_device, M, F, K, persist):
    """The fused fp8 W13 GEMM + SwiGLU + two-layout e4m3 cast (gemm_fp8_swiglu, EPI_SWIGLU_FWD8) against the unfused
    pair it replaces -- the hand fp8 GEMM on [W1; W3] then swiglu_cast_fp8_t over its gu: the same per-element
    MFMA sequence and the same gate / cast arithmetic, so gu, a8, a8t and the recorded amax must match BITWISE (random
    data), including many tiles per workgroup (persist = 40) and the Llama-1.1B width (F 5632, K 2048)."""
    h = torch.ops.bpe_hip
    torch.manual_seed(11)
    x8 = torch.randn(M, K, device=gpu_device).to(torch.float8_e4m3fn)
    w8 = (4 * torch.randn(2 * F, K, device=gpu_device)).to(torch.float8_e4m3fn)
    sp = 1.0 / (4.0 * K**0.5)  # gu ~ N(0, 1)
    sx = torch.tensor([0.25], device=gpu_device)
    sw = torch.tensor([sp / 0.25], device=gpu_device)
    sc = torch.tensor([4.0], device=gpu_device)  # the gate output's cast scale
    prev = h.gpp_persist_config(persist)
    try:
        amax_f = torch.zeros(1, dtype=torch.int32, device=gpu_device)
        a8 = torch.empty(M, F, dtype=torch.float8_e4m3fn, device=gpu_device)
        a8t = torch.empty(F, M, dtype=torch.float8_e4m3fn, device=gpu_device)
        gu = h.gemm_fp8_swiglu(x8, w8, sx, sw, sc, a8, a8t, amax_f)
        gu_ref = h.gemm_fp8(x8, w8, sx, sw)
    finally:
        h.gpp_persist_config(prev)
    amax_r = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    a8_r = torch.empty_like(a8)
    a8t_r = torch.empty_like(a8t)
    h.swiglu_cast_fp8_t(gu_ref, None, sc, a8_r, a8t_r, amax_r)
    assert torch.equal(gu, gu_ref)
    assert torch.equal(a8.view(torch.uint8), a8_r.view(torch.uint8))
    assert torch.equal(a8t.view(torch.uint8), a8t_r.view(torch.uint8))
    assert torch.equal(a8t.view(torch.uint8), a8.view(torch.uint8).t())
    assert int(amax_f) == int(amax_r) and int(amax_f) != 0
    # and against the fp32 oracle of the gate
    ref = (x8.float() @ w8.float().t()) * (sx * sw)
    g, u = ref[:, :F], ref[:, F:]
    a = g * torch.sigmoid(g) * u
    assert rel(a8.float().cpu() / 4.0, a.cpu()) < 0.08


@pytest.mark.parametrize("M,F,K,persist", [(512, 512, 256, 1), (4096, 768, 512, 40), (1024, 5632, 2048, 1)])
def test_gemm_fp8_swiglu_bwd_matches_gemm_then_cast(gpu_device, M, F, K, persist):
    """The fused fp8 W2 input gradient + SwiGLU backward + two-layout e5m2 cast (gemm_fp8_swiglu_bwd,
    EPI_SWIGLU_BWD8) against the pair it replaces -- the hand fp8 GEMM da = g8 @ w8t^T (e5m2 x e4m3) then
    swiglu_cast_fp8_t(gu, da): dgu8, dgu8t and the amax must match BITWISE."""
    h = torch.ops.bpe_hip
    torch.manual_seed(12)
    g8 = torch.randn(M, K, device=gpu_device).to(torch.float8_e5m2)
    w8t = (4 * torch.randn(F, K, device=gpu_device)).to(torch.float8_e4m3fn)
    gu = torch.randn(M, 2 * F, device=gpu_device).to(torch.bfloat16)
    sg = torch.tensor([0.25], device=gpu_device)
    sw = torch.tensor([1.0 / K**0.5], device=gpu_device)
    sc = torch.tensor([64.0], device=gpu_device)
    prev = h.gpp_persist_config(persist)
    try:
        amax_f = torch.zeros(1, dtype=torch.int32, device=gpu_device)
        d8 = torch.empty(M, 2 * F, dtype=torch.float8_e5m2, device=gpu_device)
        d8t = torch.empty(2 * F, M, dtype=torch.float8_e5m2, device=gpu_device)
        h.gemm_fp8_swiglu_bwd(g8, w8t, sg, sw, gu, sc, d8, d8t, amax_f)
        da = h.gemm_fp8(g8, w8t, sg, sw)
    finally:
        h.gpp_persist_config(prev)
    amax_r = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    d8_r = torch.empty_like(d8)
    d8t_r = torch.empty_like(d8t)
    h.swiglu_cast_fp8_t(gu, da, sc, d8_r, d8t_r, amax_r)
    assert torch.equal(d8.view(torch.uint8), d8_r.view(torch.uint8))
    assert torch.equal(d8t.view(torch.uint8), d8t_r.view(torch.uint8))
    assert torch.equal(d8t.view(torch.uint8), d8.view(torch.uint8).t())
    assert int(amax_f) == int(amax_r) and int(amax_f) != 0


def test_gemm_fp8_persistent_bitwise_many_tiles(gpu_device):
    """The fp8 kernels at production tile counts (640 output tiles: every persistent workgroup walks 2-3 of them, the
    3-workgroup form ~213), on small-integer operands whose products are exact: the one-tile, persistent and
    3-workgroup forms of gemm_fp8 and gemm_fp8_rope, and the split-K gemm_fp8_acc (160 tiles x 4 splits), must all
    equal the exact reference bitwise, on repeated runs -- a race in the seam prefetch or the store overlap (the
    bf16 persistent kernel had one, docs/performance.md) shows as wrong tiles."""
    from bpe_transformer.ops import reference as R
    h = torch.ops.bpe_hip
    g = torch.Generator(device="cpu").manual_seed(17)
    M, N, K = 16384, 2560, 1024  # 64 x 10 = 640 tiles, 8 fp8 K-tiles
    a = torch.randint(-4, 5, (M, K), generator=g).float()
    b = torch.randint(-4, 5, (N, K), generator=g).float()
    a8 = a.to(torch.float8_e4m3fn).to(gpu_device)
    b8 = b.to(torch.float8_e4m3fn).to(gpu_device)
    sa = torch.tensor([0.25], device=gpu_device)
    sb = torch.tensor([2.0], device=gpu_device)
    exact = (a.to(gpu_device) @ b.to(gpu_device).t()) * 0.5  # |sum| <= 16 K: exact in fp32
    ref = exact.to(torch.bfloat16)
    S, D, H, Hkv = 1024, 128, 12, 4  # N = (12 + 2 * 4) * 128 = 2560; RoPE on Q / K, V untouched
    cos, sin = R.rope_tables(D, S, 10000.0, device=gpu_device)
    ref_rope = ref.clone()
    h.rope_qk_(ref_rope, cos, sin, M // S, S, H, Hkv, D)
    prev, prev_o = h.gpp_persist_config(0), h.gpp_order_config(-1)
    try:
        for mode in (0, 1, 3, 1, 1):
            h.gpp_persist_config(mode)
            for gm in (0, 2, 4):  # explicit tile orders (the fp8 GEMMs are row-major in auto mode)
                h.gpp_order_config(gm)
                assert torch.equal(h.gemm_fp8(a8, b8, sa, sb), ref), (mode, gm)
                assert torch.equal(h.gemm_fp8_rope(a8, b8, sa, sb, cos, sin, S, D, (H + Hkv) * D), ref_rope), (mode, gm)
    finally:
        h.gpp_persist_config(prev)
        h.gpp_order_config(prev_o)
    # split-K weight-gradient form: 16 x 10 output tiles x 4 splits over K = 16384 tokens, fp32 C, beta = 1
    Mw, Kw = 4096, 16384
    aw = torch.randint(-2, 3, (Mw, Kw), generator=g).float()
    bw = torch.randint(-2, 3, (N, Kw), generator=g).float()
    aw8 = aw.to(torch.float8_e5m2).to(gpu_device)
    bw8 = bw.to(torch.float8_e4m3fn).to(gpu_device)
    c0 = torch.randint(-8, 9, (Mw, N), generator=g).float().to(gpu_device)
    refw = c0 + (aw.to(gpu_device) @ bw.to(gpu_device).t()) * 0.5  # |sum| <= 4 * 16384: exact in fp32
    for _ in range(3):
        c = c0.clone()
        h.gemm_fp8_acc(aw8, bw8, sa, sb, c, 1.0, 4)
        assert torch.equal(c, refw)


def test_gemm_fp8_random_vs_dequantised(gpu_device, gpp_mode):
    """Random e4m3 operands at a Llama projection shape against the fp32 product of the dequantised operands."""
    torch.manual_seed(7)
    M, N, K = 1024, 2560, 2048
    a8 = (torch.randn(M, K, device=gpu_device) * 2).to(torch.float8_e4m3fn)
    b8 = (torch.randn(N, K, device=gpu_device) * 2).to(torch.float8_e4m3fn)
    sa = torch.tensor([0.125], device=gpu_device)
    sb = torch.tensor([0.0625], device=gpu_device)
    y = torch.ops.bpe_hip.gemm_fp8(a8, b8, sa, sb)
    ref = (a8.float() @ b8.float().t()) * (0.125 * 0.0625)
    assert rel(y.float(), ref) < 5e-3


# ---------------------------------------------------------------- fp32 gradient buffers (gemm.hip / gemm_pp.hip)
@pytest.mark.parametrize("kernel,tile", [("pp", 0), ("gemm", 256), ("gemm", 128)])
@pytest.mark.parametrize("splits", [1, 4])
def test_gemm_fp32_output_accumulates_unrounded(gpu_device, kernel, tile, splits):
    """dW kernels writing an fp32 C (an fp32 gradient buffer): C = beta * C + dY^T X through the fp32 partial slab
    and the ordered reduce -- exact on small-integer operands, including a C value no bf16 can hold."""
    torch.manual_seed(2)
    N, K, T = 512, 256, 4096
    dy = torch.randint(-2, 3, (T, N), device=gpu_device).to(torch.bfloat16)
    x = torch.randint(-2, 3, (T, K), device=gpu_device).to(torch.bfloat16)
    C = torch.randint(-3, 4, (N, K), device=gpu_device).float() + 1.0 / 256  # not representable in bf16
    ref = C.double() + dy.double().t() @ x.double()
    if kernel == "pp":
        torch.ops.bpe_hip.gemm_pp(dy, False, x, False, C, 1.0, splits)
    else:
        torch.ops.bpe_hip.gemm(dy, False, x, False, C, 1.0, splits, tile)
    assert torch.equal(C.double().cpu(), ref.cpu())


def test_accumulate_weight_grad_fp32_buffer(gpu_device):
    """The dW route with an fp32 gradient view (TrainEngine(grad_dtype=fp32)): four accumulations stay within
    fp32 rounding of the fp64 sum, where a bf16 buffer is off by its own rounding."""
    from bpe_transformer.ops.gemm import accumulate_weight_grad

    torch.manual_seed(3)
    T, N, K = 8192, 768, 768
    g32 = torch.zeros(N, K, device=gpu_device)
    g16 = torch.zeros(N, K, device=gpu_device, dtype=torch.bfloat16)
    ref = torch.zeros(N, K, device=gpu_device, dtype=torch.float64)
    for _ in range(4):
        dy = torch.randn(T, N, device=gpu_device, dtype=torch.bfloat16)
        x = torch.randn(T, K, device=gpu_device, dtype=torch.bfloat16)
        accumulate_weight_grad(g32, dy, x)
        accumulate_weight_grad(g16, dy, x)
        ref += dy.double().t() @ x.double()
    e32 = float((g32.double() - ref).norm() / ref.norm())
    e16 = float((g16.double() - ref).norm() / ref.norm())
    assert e32 < 1e-6 and e16 > 100 * e32, (e32, e16)


@pytest.mark.parametrize("S,H,Hkv,causal", [(1024, 4, 4, True), (200, 8, 2, True), (1000, 4, 4, False), (64, 2, 2, True),
                                            (600, 2, 2, True)])
def test_flash_fwd_v4_matches_v2_and_oracle(gpu_device, S, H, Hkv, causal):
    """The D = 64 forward v8 (running max in the S accumulator's start, row sum by MFMA, no tile max on the common
    path) against fa_fwd_kernel (v2) on the same inputs and against the fp32 oracle: O and the base-2 LSE."""
    h = torch.ops.bpe_hip
    B, D = 2, 64
    torch.manual_seed(21)
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device=gpu_device, dtype=torch.bfloat16)
    qkv[:, : H * D] *= 2.0
    q, k, v = qkv[:, : H * D], qkv[:, H * D : (H + Hkv) * D], qkv[:, (H + Hkv) * D :]
    e = torch.empty(0, 0, device=gpu_device)
    prev = h.fa_fwd_config(8)
    try:
        o4, l4 = h.fa_fwd(q, k, v, e, e, B, S, H, Hkv, D, causal, False, D ** -0.5, False)
        h.fa_fwd_config(2)
        o2, l2 = h.fa_fwd(q, k, v, e, e, B, S, H, Hkv, D, causal, False, D ** -0.5, False)
    finally:
        h.fa_fwd_config(prev)
    orf = ops.attention_qkv_reference(qkv.float().cpu(), B, S, H, Hkv, D, None, None, causal)
    e4, e2 = rel(o4.float().cpu(), orf), rel(o2.float().cpu(), orf)
    assert e4 < 1e-2 and e4 < 1.5 * e2 + 1e-3, (e4, e2)
    # v4's row sum is the MFMA sum of the bf16-rounded P that O accumulates (v2 adds the fp32 P): rows with few
    # keys differ by up to ~one bf16 rounding of P, 2^-9 -> 0.003 in log2 units
    assert torch.allclose(l4, l2, atol=6e-3, rtol=1e-4), float((l4 - l2).abs().max())


# ---------------------------------------------------------------- generic masked SDPA (contract K7, csrc/masked_sdpa.hip)
def test_sdpa_contract_snapshots_on_gpu(gpu_device, q, k, v, mask):
    """The reference's own SDPA snapshots (``tests/_snapshots/test_{,4d_}scaled_dot_product_attention.npz``,
    ``/root/reference/tests/test_model.py:57-74``, atol 1e-6) with GPU inputs: the adapter runs the HIP kernel."""
    from .adapters import run_scaled_dot_product_attention
    from .conftest import NumpySnapshot

    qg, kg, vg, mg = (t.to(gpu_device) for t in (q, k, v, mask))
    out = run_scaled_dot_product_attention(qg, kg, vg, mg)
    assert out.is_cuda
    NumpySnapshot("test_scaled_dot_product_attention", False).assert_match(out, atol=1e-6)
    q4, k4, v4, m4 = (t.reshape(2, 2, *t.shape[1:]) for t in (qg, kg, vg, mg))
    out4 = run_scaled_dot_product_attention(q4, k4, v4, m4)
    NumpySnapshot("test_4d_scaled_dot_product_attention", False).assert_match(out4, atol=1e-6)


def test_masked_sdpa_many_batch_heads_falls_back(gpu_device):
    """More batch-heads than the kernel's grid.y (65535) take the oracle path instead of failing; an int mask counts
    nonzero as attend there too."""
    torch.manual_seed(3)
    Q = torch.randn(65536 + 7, 2, 8, device=gpu_device)
    K = torch.randn(65536 + 7, 3, 8, device=gpu_device)
    V = torch.randn(65536 + 7, 3, 8, device=gpu_device)
    m = torch.tensor([[1, 1, 0], [1, 0, 1]], device=gpu_device)
    got = ops.scaled_dot_product_attention(Q, K, V, m)
    ref = R.scaled_dot_product_attention(Q.float(), K.float(), V.float(), m.bool())
    assert got.shape == ref.shape and rel(got, ref) < 1e-5


@pytest.mark.parametrize("lead,Sq,Sk,D,Dv", [((3,), 7, 5, 16, 16), ((2, 3), 70, 130, 64, 32), ((1,), 129, 64, 128, 128),
                                            ((4, 2), 33, 200, 24, 100)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mask_kind", ["none", "full", "broadcast_qk", "causal"])
def test_masked_sdpa_vs_oracle(gpu_device, lead, Sq, Sk, D, Dv, dtype, mask_kind):
    """Random shapes (tiles of 64 keys with ragged tails, head dims 16..128, Dv != D), fp32 and bf16 operands, and
    masks given per (lead, q, k), broadcast over the leading dims, or none -- against the fp32 oracle."""
    torch.manual_seed(9)
    Q = torch.randn(*lead, Sq, D, device=gpu_device).to(dtype)
    K = torch.randn(*lead, Sk, D, device=gpu_device).to(dtype)
    V = torch.randn(*lead, Sk, Dv, device=gpu_device).to(dtype)
    m = None
    if mask_kind == "full":
        m = torch.rand(*lead, Sq, Sk, device=gpu_device) > 0.3
        m[..., 0] = True  # every row attends to something (all-masked rows: the next test)
    elif mask_kind == "broadcast_qk":
        m = torch.rand(Sq, Sk, device=gpu_device) > 0.3
        m[..., 0] = True
    elif mask_kind == "causal":
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=gpu_device).tril()
    got = ops.scaled_dot_product_attention(Q, K, V, m)
    ref = ops.reference.scaled_dot_product_attention(Q.float().cpu(), K.float().cpu(), V.float().cpu(),
                                                     None if m is None else m.cpu())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert got.dtype == dtype and got.shape == ref.shape
    err = float((got.float().cpu() - ref).abs().max())
    assert err < tol, err


def test_masked_sdpa_all_masked_row_is_nan_and_grad(gpu_device):
    """A row with every key masked is NaN (softmax over all -inf, as the oracle); gradients flow through the
    autograd wrapper (oracle-formula backward) and match the oracle's."""
    torch.manual_seed(2)
    Q, K, V = (torch.randn(2, 9, 32, device=gpu_device) for _ in range(3))
    m = torch.rand(2, 9, 9, device=gpu_device) > 0.5
    m[:, :, 0] = True
    m[1, 4] = False
    out = ops.scaled_dot_product_attention(Q, K, V, m)
    assert torch.isnan(out[1, 4]).all() and not torch.isnan(out[0]).any() and not torch.isnan(out[1, 5:]).any()
    m[1, 4, 0] = True
    Qg, Kg, Vg = (t.clone().requires_grad_(True) for t in (Q, K, V))
    d = torch.randn(2, 9, 32, device=gpu_device)
    (ops.scaled_dot_product_attention(Qg, Kg, Vg, m) * d).sum().backward()
    Qr, Kr, Vr = (t.cpu().requires_grad_(True) for t in (Q, K, V))
    (ops.reference.scaled_dot_product_attention(Qr, Kr, Vr, m.cpu()) * d.cpu()).sum().backward()
    for g, gr in ((Qg.grad, Qr.grad), (Kg.grad, Kr.grad), (Vg.grad, Vr.grad)):
        assert float((g.cpu() - gr).abs().max()) < 1e-4
