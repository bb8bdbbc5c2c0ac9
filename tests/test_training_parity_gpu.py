"""At-scale training parity: the fused HIP training engine against an independent eager PyTorch implementation.

The reference implies one training step (``/root/reference/tests/test_optimizer.py:18-25``: forward, cross-entropy,
backward, clip, AdamW with a cosine schedule).  Here both implementations train the same model from identical
weights on the same real-token batches for 150 steps:

* ours: ``TrainEngine`` -- bf16 weights, fp32 master and moments in the flat AdamW kernel, fused blocks (split
  flash attention, SwiGLU GEMM epilogues, TN-layout input gradients), fused LM head + CE, device-side clip;
* eager: a separate module tree written here with ``torch.nn.functional.scaled_dot_product_attention`` (KV heads
  repeated for GQA), fp32 parameters under bf16 autocast, ``torch.optim.AdamW``, ``clip_grad_norm_`` and the same
  cosine schedule.

Shapes (2 layers each, so the tests stay short):

* ``gpt2``: d_model 768, 12 heads, SwiGLU d_ff 2048, batch x seq = 4 x 1024 -- with one micro-batch per step and
  with 4 accumulated micro-batches (fp32 gradient buffer);
* ``llama``: d_model 2048, 32 query / 4 KV heads (GQA, the split backward's KV-head sweep), d_ff 5632 (the
  unfused SwiGLU forward past d_model 1024), batch x seq = 2 x 2048;
* ``d128``: d_model 1024, 8 query / 2 KV heads of 128 (the split backward at D = 128), d_ff 2816, 2 x 2048;
* ``llama`` fp8: our engine with fp8 projections (e4m3 forward, e5m2 x e4m3 input gradients) against our bf16
  engine, once through the per-shape routes and once with every fp8 GEMM forced onto the hand-written
  ``gemm_pp`` F8 kernel (``BPE_FP8_GEMM=hip``).

Tokens: a 4 096-token BPE vocabulary trained here (``train_bpe``) on ``tinystories_sample.txt``, encoding
``corpus.en`` + ``tinystories_sample.txt`` (the reference's pickled sample tokenizer is not shipped to the GPU box).
Set ``BPE_PARITY_LOG=<dir>`` to write the loss curves.
"""

from __future__ import annotations

import functools
import json
import math
import os
from dataclasses import dataclass

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from .conftest import FIXTURES

pytestmark = pytest.mark.gpu

STEPS, L, THETA = 150, 2, 10000.0
WARMUP = 10


@dataclass(frozen=True)
class Shape:
    name: str
    B: int
    S: int
    D: int
    H: int
    Hkv: int
    FF: int
    lr: float  # peak learning rate (cosine to lr / 10)


# Llama-shape peak LR 3e-4 (the usual for d_model 2048): at 1e-3 both implementations hit loss spikes from step ~25
# on and their trajectories part chaotically (matching to 6e-4 relative before the first spike), which says nothing
# about the arithmetic.
SHAPES = {"gpt2": Shape("gpt2shape", 4, 1024, 768, 12, 12, 2048, 1e-3),
          "llama": Shape("llamashape", 2, 2048, 2048, 32, 4, 5632, 3e-4),
          # head size 128 (the D = 128 split backward, RoPE in the QKV GEMM epilogue), GQA 8:2
          "d128": Shape("headdim128", 2, 2048, 1024, 8, 2, 2816, 5e-4)}


def _lr(it: int, c) -> float:
    from bpe_transformer.optim.schedule import get_lr_cosine_schedule

    return get_lr_cosine_schedule(it, c.lr, c.lr / 10, WARMUP, STEPS)


class _RMS(nn.Module):
    def __init__(self, d, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x):
        xf = x.float()
        return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps) * self.weight.float()


def _rope(x, cos, sin):  # x [B, H, S, Dh], interleaved pairs (2i, 2i+1)
    x1, x2 = x[..., 0::2].float(), x[..., 1::2].float()
    out = torch.stack((x1 * cos - x2 * sin, x1 * sin + x2 * cos), dim=-1)
    return out.flatten(-2).to(x.dtype)


class _Attn(nn.Module):
    def __init__(self, c: Shape):
        super().__init__()
        self.c = c
        dk = c.D // c.H
        self.q_proj = nn.Linear(c.D, c.D, bias=False)
        self.k_proj = nn.Linear(c.D, c.Hkv * dk, bias=False)
        self.v_proj = nn.Linear(c.D, c.Hkv * dk, bias=False)
        self.output_proj = nn.Linear(c.D, c.D, bias=False)

    def forward(self, x, cos, sin):
        b, s, _ = x.shape
        c, dk = self.c, self.c.D // self.c.H
        q = self.q_proj(x).view(b, s, c.H, dk).transpose(1, 2)
        k, v = (p(x).view(b, s, c.Hkv, dk).transpose(1, 2) for p in (self.k_proj, self.v_proj))
        q, k = _rope(q, cos, sin), _rope(k, cos, sin)
        if c.Hkv < c.H:  # GQA: query head h reads KV head h // (H / Hkv)
            k, v = (t.repeat_interleave(c.H // c.Hkv, dim=1) for t in (k, v))
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.output_proj(o.transpose(1, 2).reshape(b, s, c.D))


class _FFN(nn.Module):
    def __init__(self, c: Shape):
        super().__init__()
        self.w1 = nn.Linear(c.D, c.FF, bias=False)
        self.w2 = nn.Linear(c.FF, c.D, bias=False)
        self.w3 = nn.Linear(c.D, c.FF, bias=False)

    def forward(self, x):
        return self.w2(F.silu(self.w1(x)) * self.w3(x))


class _Block(nn.Module):
    def __init__(self, c: Shape):
        super().__init__()
        self.ln1, self.attn, self.ln2, self.ffn = _RMS(c.D), _Attn(c), _RMS(c.D), _FFN(c)

    def forward(self, x, cos, sin):
        x = x + self.attn(self.ln1(x), cos, sin)
        return x + self.ffn(self.ln2(x))


class EagerLM(nn.Module):
    """Independent implementation with the reference's parameter names (``tests/adapters.py:311-353``)."""

    def __init__(self, vocab, c: Shape):
        super().__init__()
        D, H, S = c.D, c.H, c.S
        self.token_embeddings = nn.Embedding(vocab, D)
        self.layers = nn.ModuleList(_Block(c) for _ in range(L))
        self.ln_final = _RMS(D)
        self.lm_head = nn.Linear(D, vocab, bias=False)
        inv = THETA ** (-torch.arange(0, D // H, 2, dtype=torch.float64) / (D // H))
        ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None, :]
        self.register_buffer("cos", ang.cos().float(), persistent=False)
        self.register_buffer("sin", ang.sin().float(), persistent=False)

    def loss(self, x, y):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            h = self.token_embeddings(x)
            for blk in self.layers:
                h = blk(h, self.cos, self.sin)
            logits = self.lm_head(self.ln_final(h))
        return F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), y.reshape(-1))


@pytest.fixture(autouse=True)
def _fixed_dw_routes(monkeypatch):
    """The dW route of a shape missing from ops/tuning/dw_routes.json is otherwise timed on first use (ops/gemm.py),
    so two runs could take different kernels -- different bf16 roundings that a 150-step trajectory amplifies.
    Here every off-table shape takes its first candidate, from a fresh route cache."""
    from bpe_transformer.ops import gemm

    monkeypatch.setattr(gemm, "_AUTOTUNE", False)
    monkeypatch.setattr(gemm, "_route", {})


@functools.lru_cache(maxsize=1)
def _tokens():
    from bpe_transformer import train_bpe
    from bpe_transformer.tokenization import BPETokenizer

    vocab, merges = train_bpe(str(FIXTURES / "tinystories_sample.txt"), 4096, ["<|endoftext|>"])
    tok = BPETokenizer(vocab, merges, ["<|endoftext|>"])
    text = (FIXTURES / "corpus.en").read_text(encoding="utf-8") + "<|endoftext|>"
    text += (FIXTURES / "tinystories_sample.txt").read_text(encoding="utf-8") * 8
    return torch.tensor(tok.encode(text), dtype=torch.long), len(tok.vocab)


def _batches(ids, n, micro, S, dev):
    g = torch.Generator().manual_seed(1234)
    out = []
    for _ in range(n):
        st = torch.randint(0, ids.numel() - S - 1, (micro,), generator=g)
        w = torch.stack([ids[s : s + S + 1] for s in st.tolist()]).to(dev)
        out.append((w[:, :-1].contiguous(), w[:, 1:].contiguous()))
    return out


def _ours(vocab, c: Shape, dev):
    from bpe_transformer.models import TransformerLM

    torch.manual_seed(0)
    return TransformerLM(vocab, c.S, c.D, L, c.H, c.FF, THETA, num_kv_heads=c.Hkv, device=dev, dtype=torch.bfloat16)


def _engine(model, accum, c):
    from bpe_transformer.train.engine import TrainEngine

    return TrainEngine(model, lr=c.lr, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0,
                       grad_dtype=torch.float32 if accum > 1 else None)


def _run(c: Shape, accum: int, gpu_device):
    """Our engine vs the eager implementation: (our losses, eager losses)."""
    assert torch.ops.bpe_hip.fa_bwd_config(-1) == 0, "the default D = 64 backward is the split form"
    ids, vocab = _tokens()
    ours = _ours(vocab, c, gpu_device)
    eager = EagerLM(vocab, c).to(gpu_device)
    missing, unexpected = eager.load_state_dict({k: v.float() for k, v in ours.state_dict().items()}, strict=False)
    assert not missing and not [k for k in unexpected if "rope" not in k], (missing, unexpected)
    eng = _engine(ours, accum, c)
    decay = [p for p in eager.parameters() if p.dim() >= 2]
    nodecay = [p for p in eager.parameters() if p.dim() < 2]
    opt = torch.optim.AdamW([{"params": decay, "weight_decay": 0.1}, {"params": nodecay, "weight_decay": 0.0}],
                            lr=c.lr, betas=(0.9, 0.95), eps=1e-8)
    micro = c.B // accum
    data = _batches(ids, STEPS * accum, micro, c.S, gpu_device)
    lo, le = [], []
    for it in range(STEPS):
        mb = data[it * accum : (it + 1) * accum]
        lo.append(eng.train_step(mb, lr=_lr(it, c)))
        lr = _lr(it, c)
        for gr in opt.param_groups:
            gr["lr"] = lr
        opt.zero_grad(set_to_none=True)
        tot = 0.0
        for x, y in mb:
            loss = eager.loss(x, y)
            (loss / accum).backward()
            tot += loss.detach()
        torch.nn.utils.clip_grad_norm_(eager.parameters(), 1.0)
        opt.step()
        le.append(tot / accum)
    lo = [float(v) for v in torch.stack(lo).cpu()]
    le = [float(v) for v in torch.stack(le).cpu()]
    return lo, le


def _run_ours(c: Shape, fp8: bool, gpu_device, wgrad: bool = True):
    ids, vocab = _tokens()
    model = _ours(vocab, c, gpu_device)
    if fp8:
        model.enable_fp8(wgrad=wgrad)
    eng = _engine(model, 1, c)
    data = _batches(ids, STEPS, c.B, c.S, gpu_device)
    out = [eng.train_step([data[it]], lr=_lr(it, c)) for it in range(STEPS)]
    return [float(v) for v in torch.stack(out).cpu()]


def _log(name, payload):
    log = os.environ.get("BPE_PARITY_LOG")
    if log:
        os.makedirs(log, exist_ok=True)
        with open(os.path.join(log, name), "w") as f:
            json.dump(payload, f)


@pytest.mark.parametrize("shape,accum", [("gpt2", 1), ("gpt2", 4), ("llama", 1), ("d128", 1)])
def test_fused_engine_tracks_eager_pytorch(gpu_device, shape, accum):
    c = SHAPES[shape]
    lo, le = _run(c, accum, gpu_device)
    assert all(math.isfinite(v) for v in lo + le)
    rel = [abs(a - b) / b for a, b in zip(lo, le)]
    _log(f"parity_{c.name}_L{L}_accum{accum}.json",
         {"steps": STEPS, "batch": c.B, "seq": c.S, "d_model": c.D, "heads": c.H, "kv_heads": c.Hkv, "d_ff": c.FF,
          "accum": accum, "ours": lo, "eager": le, "max_rel": max(rel), "final_rel": rel[-1]})
    assert le[-1] < le[0] - 2.0, "the eager reference did not learn: the comparison would be vacuous"
    assert lo[-1] < lo[0] - 2.0
    assert max(rel) < 0.02, (max(rel), rel.index(max(rel)))
    assert rel[-1] < 0.01, rel[-1]


@pytest.mark.parametrize("route,wgrad", [("routes", True), ("hip", True), ("routes", False)])
def test_fp8_engine_tracks_bf16_engine(gpu_device, monkeypatch, route, wgrad):
    """fp8 projections (``model.enable_fp8()``: delayed-scaling e4m3 / e5m2, ops/fp8.py) against the bf16 engine on
    the Llama shape: the final loss within 2 %, the 10-step running mean within 3 % throughout with bf16 weight
    gradients and within 4 % with fp8 ones (single steps of the early transient differ by more: the two precisions
    take different paths through the same loss landscape; the e5m2 rounding of the gradient in dW widens the
    transient -- measured 1.5 % vs 3.0 % at its peak -- while the final loss stays within 1.01 %, e5m2 margin 2;
    single-step gaps of up to 27 % are the two trajectories' weights: test_fp8_forward_matches_bf16_on_same_weights).
    ``route``: the per-shape route table, or every fp8 GEMM on the hand-written gemm_pp F8 kernel (asserted: the
    hand kernel served every fp8 GEMM of the run -- forward, input and weight gradients at this 4096-token shape)."""
    from bpe_transformer.ops import fp8

    monkeypatch.setattr(fp8, "_MODE", route)
    taken = {True: 0, False: 0}
    use_hip = fp8._use_hip

    def counted(*a):
        r = use_hip(*a)
        taken[r] += 1
        return r

    monkeypatch.setattr(fp8, "_use_hip", counted)
    c = SHAPES["llama"]
    lb = _run_ours(c, False, gpu_device)
    l8 = _run_ours(c, True, gpu_device, wgrad)
    if route == "hip":
        assert taken[True] > 0 and taken[False] == 0, taken
    assert all(math.isfinite(v) for v in lb + l8)
    rel = [abs(a - b) / b for a, b in zip(l8, lb)]
    run = lambda x: [sum(x[max(0, i - 9) : i + 1]) / len(x[max(0, i - 9) : i + 1]) for i in range(len(x))]  # noqa: E731
    rel_mean = [abs(a - b) / b for a, b in zip(run(l8), run(lb))]
    _log(f"parity_{c.name}_L{L}_fp8_{route}{'' if wgrad else '_bf16wgrad'}_vs_bf16.json",
         {"steps": STEPS, "batch": c.B, "seq": c.S, "route": route, "fp8_wgrad": wgrad, "fp8": l8, "bf16": lb,
          "max_rel": max(rel), "max_rel_mean10": max(rel_mean), "final_rel": rel[-1], "gemm_fp8_calls": taken})
    assert lb[-1] < lb[0] - 2.0
    assert max(rel_mean) < (0.04 if wgrad else 0.03), (max(rel_mean), rel_mean.index(max(rel_mean)))
    assert rel[-1] < 0.02, rel[-1]


def _same_weights_losses(c: Shape, steps, gpu_device, margin: float = 1.0, train: bool = False) -> dict:
    """Train the bf16 engine and, before step s in ``steps``, evaluate batch s on the SAME weights in bf16 and in fp8
    (scales calibrated on the 16 preceding batches, what the delayed recipe holds at that step).

    ``train``: evaluate with gradients enabled (no backward, no optimizer step), so the fused block takes its
    TRAINING forward -- with fp8 weight gradients the two RMSNorms write h1 / h2 only as e4m3 in both layouts
    (``add_rmsnorm_cast_t``) and the gate writes a only as e4m3 (``swiglu_fwd_cast_t``, or the fused W13 GEMM's
    epilogue, ``matmul_swiglu``), kernels an eval-mode forward never runs."""
    ids, vocab = _tokens()
    model = _ours(vocab, c, gpu_device)
    eng = _engine(model, 1, c)
    data = _batches(ids, STEPS, c.B, c.S, gpu_device)
    out = {}
    for it in range(max(steps) + 1):
        if it in steps:
            with torch.set_grad_enabled(train):
                x, y = data[it]
                lb = float(model.loss(x, y).detach())
                model.enable_fp8(margin=margin, wgrad=True if train else None)
                for jt in range(max(0, it - 16), it):
                    model.loss(*data[jt]).detach()
                    for st in model.fp8_states():
                        st.update()
                l8 = float(model.loss(x, y).detach())
                for layer in model.layers:
                    layer.fp8 = None
                model.fp8_state = model.fp8_grad_state = None
            out[it] = (lb, l8)
        eng.train_step([data[it]], lr=_lr(it, c))
    return out


def test_fp8_forward_matches_bf16_on_same_weights(gpu_device, monkeypatch):
    """Per-step bound on the fp8 TRAINING forward itself: at the steps where the fp8 run's loss departs most from the
    bf16 run's (18, 25, 73: up to 27 %, benchmarks/fp8_spike_probe.py), the fp8 forward on the bf16 run's own weights
    -- evaluated with gradients enabled, so through the kernels a training step runs (the fused norm + e4m3 casts
    and the gate + e4m3 cast, counted here) -- is within 1 % of the bf16 forward.  The transient gaps of
    test_fp8_engine_tracks_bf16_engine are therefore the two trajectories' weights, not the rounding of one fp8
    step (profiles/parity/fp8_spike_probe_r5.json)."""
    from bpe_transformer.models import fused_block as fb

    ran = {"norm8": 0, "swiglu_cast": 0, "swiglu_gemm": 0}

    def counted(name, fn):
        def f(*a, **k):
            ran[name] += 1
            return fn(*a, **k)
        return f

    monkeypatch.setattr(fb, "add_rmsnorm_cast_t", counted("norm8", fb.add_rmsnorm_cast_t))
    monkeypatch.setattr(fb, "swiglu_fwd_cast_t", counted("swiglu_cast", fb.swiglu_fwd_cast_t))
    # the gate's e4m3 cast runs either as its own pass or, by default, in the fused fp8 W13 GEMM's epilogue
    monkeypatch.setattr(fb, "matmul_swiglu", counted("swiglu_gemm", fb.matmul_swiglu))
    res = _same_weights_losses(SHAPES["llama"], [18, 25, 73], gpu_device, train=True)
    _log("parity_llamashape_L2_fp8_same_weights.json", {str(k): {"bf16": v[0], "fp8": v[1]} for k, v in res.items()})
    assert ran["norm8"] > 0 and ran["swiglu_cast"] + ran["swiglu_gemm"] > 0, ran
    for it, (lb, l8) in res.items():
        assert math.isfinite(l8) and abs(l8 - lb) / lb < 0.01, (it, lb, l8)
