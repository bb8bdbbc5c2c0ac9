"""Serving benchmark: KV-cache decode throughput / latency (``models/generation.py``).

For each batch size: prefill a prompt, then time ``--tokens`` decode steps (HIP-graph replay by default,
``--no-graph`` for eager launches), and the decode-attention kernel alone at the final cache length (HBM
bandwidth of the K/V read).  ``--recompute`` also times the cache-less baseline (full prefix re-run per token).
Random-init weights, synthetic prompts; one JSON line per configuration.

    python benchmarks/decode_bench.py --model gpt2-small --batch 1 8 64 --prompt 128 --tokens 256
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.models import DecodeSession, TransformerLM, get_preset  # noqa: E402
from bpe_transformer.ops import decode as dec  # noqa: E402


def time_decode(sess, ids, prompt_len, tokens):
    sess.reset()
    sess.prefill(ids[:, :prompt_len])
    nxt = ids[:, prompt_len]
    sess.decode(nxt)  # graph capture / first-use costs outside the timed loop
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(tokens):
        sess.decode(nxt)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / tokens


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8, 64])
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--recompute", action="store_true")
    a = ap.parse_args()
    cfg = get_preset(a.model)
    torch.manual_seed(0)
    model = TransformerLM.from_config(cfg, device="cuda", dtype=torch.bfloat16).eval()
    max_len = a.prompt + a.tokens + 2
    for B in a.batch:
        ids = torch.randint(0, cfg.vocab_size, (B, a.prompt + 1), device="cuda")
        sess = DecodeSession(model, B, max_len=max_len, use_graph=not a.no_graph)
        with torch.no_grad():
            # prefill throughput
            sess.reset()
            sess.prefill(ids[:, : a.prompt])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                sess.reset()
                sess.prefill(ids[:, : a.prompt])
            torch.cuda.synchronize()
            t_pre = (time.perf_counter() - t0) / 3
            t_tok = time_decode(sess, ids, a.prompt, a.tokens)
            # the attention kernel alone at the final length (all layers' worth of K/V bytes per call)
            L = sess.length
            q = torch.randn(B, sess.H * sess.D, device="cuda", dtype=torch.bfloat16)
            pos = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
            kc, vc = sess.cache.k[0], sess.cache.v[0]
            for _ in range(3):
                dec.decode_attention(q, kc, vc, pos, sess.H)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                dec.decode_attention(q, kc, vc, pos, sess.H)
            e1.record()
            torch.cuda.synchronize()
            t_attn = e0.elapsed_time(e1) / 50 / 1e3
            kv_bytes = 2 * B * sess.Hkv * L * sess.D * 2
            out = {
                "model": a.model, "batch": B, "prompt": a.prompt, "decode_tokens": a.tokens,
                "graph": not a.no_graph,
                "prefill_ms": round(t_pre * 1e3, 3),
                "prefill_tok_s": round(B * a.prompt / t_pre, 1),
                "decode_ms_per_step": round(t_tok * 1e3, 4),
                "decode_tok_s": round(B / t_tok, 1),
                "attn_us_per_layer": round(t_attn * 1e6, 2),
                "attn_kv_GBps": round(kv_bytes / t_attn / 1e9, 1),
                "cache_len": L,
            }
            if a.recompute:
                n = 16
                ctx = ids[:, : a.prompt]
                model(ctx)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(n):
                    model(ctx)[:, -1].argmax(-1)
                torch.cuda.synchronize()
                out["recompute_ms_per_token"] = round((time.perf_counter() - t0) / n * 1e3, 3)
        print(json.dumps(out), flush=True)
        del sess
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
