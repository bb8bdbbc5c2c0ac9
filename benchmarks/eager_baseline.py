"""The BASELINE.md comparison point: the same GPT-2-small-shape model written as a plain PyTorch eager
program (no HIP kernels, no fusion, no flat buffers), trained on the same synthetic data.

    python benchmarks/eager_baseline.py --attn sdpa   # F.scaled_dot_product_attention (library flash path)
    python benchmarks/eager_baseline.py --attn naive  # explicit QK^T / mask / softmax / PV

Architecture = ``bpe_transformer.models.TransformerLM`` (pre-norm RMSNorm, interleaved RoPE, causal MHA,
SwiGLU, untied LM head); mixed precision the usual eager way: fp32 parameters, ``torch.autocast`` bf16,
``torch.optim.AdamW(fused=True)``, grad-norm clip 1.0.  Prints one JSON line in the bench.py format.
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch import nn  # noqa: E402

from bpe_transformer.models import get_preset  # noqa: E402


class RMSNorm(nn.Module):
    def __init__(self, d, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps) * self.weight).to(x.dtype)


class Block(nn.Module):
    def __init__(self, d, h, f, attn):
        super().__init__()
        self.h, self.attn_mode = h, attn
        self.ln1, self.ln2 = RMSNorm(d), RMSNorm(d)
        self.q, self.k, self.v, self.o = (nn.Linear(d, d, bias=False) for _ in range(4))
        self.w1, self.w3 = nn.Linear(d, f, bias=False), nn.Linear(d, f, bias=False)
        self.w2 = nn.Linear(f, d, bias=False)

    @staticmethod
    def rope(x, cos, sin):  # interleaved pairs
        x1, x2 = x[..., 0::2], x[..., 1::2]
        return torch.stack((x1 * cos - x2 * sin, x1 * sin + x2 * cos), -1).flatten(-2)

    def forward(self, x, cos, sin):
        B, S, d = x.shape
        hd = d // self.h
        y = self.ln1(x)
        q, k, v = (m(y).view(B, S, self.h, hd).transpose(1, 2) for m in (self.q, self.k, self.v))
        q, k = self.rope(q, cos, sin), self.rope(k, cos, sin)
        if self.attn_mode == "sdpa":
            a = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        else:
            s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
            mask = torch.ones(S, S, dtype=torch.bool, device=x.device).tril()
            a = torch.softmax(s.masked_fill(~mask, float("-inf")).float(), -1).to(v.dtype) @ v
        x = x + self.o(a.transpose(1, 2).reshape(B, S, d))
        y = self.ln2(x)
        return x + self.w2(F.silu(self.w1(y)) * self.w3(y))


class LM(nn.Module):
    def __init__(self, cfg, attn):
        super().__init__()
        self.emb = nn.Embedding(cfg.vocab_size, cfg.d_model)
        self.blocks = nn.ModuleList(Block(cfg.d_model, cfg.num_heads, cfg.d_ff, attn) for _ in range(cfg.num_layers))
        self.ln = RMSNorm(cfg.d_model)
        self.head = nn.Linear(cfg.d_model, cfg.vocab_size, bias=False)
        hd = cfg.d_model // cfg.num_heads
        inv = cfg.rope_theta ** (-torch.arange(0, hd, 2, dtype=torch.float32) / hd)
        ang = torch.arange(cfg.context_length, dtype=torch.float32)[:, None] * inv[None]
        self.register_buffer("cos", ang.cos(), persistent=False)
        self.register_buffer("sin", ang.sin(), persistent=False)

    def forward(self, ids, tgt):
        S = ids.shape[1]
        x = self.emb(ids)
        for b in self.blocks:
            x = b(x, self.cos[:S], self.sin[:S])
        logits = self.head(self.ln(x))
        return F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), tgt.reshape(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--attn", choices=["sdpa", "naive"], default="sdpa")
    a = ap.parse_args()
    torch.manual_seed(0)
    cfg = get_preset(a.model, context_length=a.seq)
    model = LM(cfg, a.attn).cuda()
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4, weight_decay=0.1, fused=True)
    data = torch.randint(0, cfg.vocab_size, (a.batch * 8, a.seq + 1), device="cuda")

    def step(i):
        w = data[(i * a.batch) % (data.shape[0] - a.batch):][: a.batch]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = model(w[:, :-1], w[:, 1:])
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(a.warmup + i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tok = a.steps * a.batch * a.seq
    print(json.dumps({"metric": "training tokens/sec, PyTorch eager baseline", "value": round(tok / dt, 1),
                      "unit": "tokens/s", "n_gpus": 1, "ms_per_step": round(dt / a.steps * 1000, 3),
                      "attn": a.attn, "dtype": "bf16 autocast, fp32 master", "final_loss": round(loss.item(), 4),
                      "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                      "config": {"model": a.model, "batch": a.batch, "seq_len": a.seq}}), flush=True)


if __name__ == "__main__":
    main()
