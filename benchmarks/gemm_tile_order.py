"""Tile order of the one-pass ping-pong GEMMs (``gpp_order_config``): row-major against column-major bands of gm
row blocks (gemm_pp.hip ``tile_rc``), on the GPT-2 B 128 forward / SwiGLU GEMMs (131 072 tokens, K = 768).

    python benchmarks/gemm_tile_order.py [--tokens 131072] [--orders 0,2,4,8,16]

One JSON line per (GEMM, order): median ms over interleaved repetitions and whether the output is bitwise equal
to the row-major one (the order changes which workgroup computes a tile, not the tile's arithmetic).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--orders", default="0,2,4,8,16")
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--ff", type=int, default=2048)
    ap.add_argument("--nqkv", type=int, default=0, help="QKV output width (default 3 d; GQA: d + 2 kv width)")
    a = ap.parse_args()
    h = ops()
    M, d, F = a.tokens, a.d, a.ff
    orders = [int(x) for x in a.orders.split(",")]
    torch.manual_seed(0)
    x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    w13 = (0.05 * torch.randn(2 * F, d, device="cuda")).to(torch.bfloat16)
    nqkv = a.nqkv or 3 * d
    wqkv = (0.05 * torch.randn(nqkv, d, device="cuda")).to(torch.bfloat16)
    w2 = (0.05 * torch.randn(d, F, device="cuda")).to(torch.bfloat16)
    dy = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    S, D = 1024, 64
    pos = torch.arange(S, device="cuda", dtype=torch.float32)[:, None]
    inv = 10000.0 ** (-torch.arange(0, D, 2, device="cuda", dtype=torch.float32) / D)
    cos, sin = torch.cos(pos * inv), torch.sin(pos * inv)
    gu0, _ = h.gemm_swiglu_fwd(x, w13)
    c13 = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    cases = {
        "qkv_rope": lambda: h.gemm_qkv_rope(x, wqkv, cos, sin, S, D, nqkv - (nqkv - d) // 2),
        "swiglu_fwd": lambda: h.gemm_swiglu_fwd(x, w13),
        "swiglu_bwd": lambda: h.gemm_swiglu_bwd(dy, w2, gu0),
        "w13_plain": lambda: h.gemm_pp(x, True, w13, True, c13, 0.0, 1) or c13,
    }
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    prev = h.gpp_order_config(-1)
    for name, fn in cases.items():
        ref = None
        times = {o: [] for o in orders}
        same = {}
        for o in orders:  # outputs
            h.gpp_order_config(o)
            out = fn()
            out = out if isinstance(out, (tuple, list)) else (out,)
            torch.cuda.synchronize()
            if ref is None:
                ref = [t.clone() for t in out]
            same[o] = all(torch.equal(r, t) for r, t in zip(ref, out))
        for _ in range(7):  # interleaved timing
            for o in orders:
                h.gpp_order_config(o)
                fn()
                ev[0].record()
                for _ in range(3):
                    fn()
                ev[1].record()
                torch.cuda.synchronize()
                times[o].append(ev[0].elapsed_time(ev[1]) / 3)
        for o in orders:
            print(json.dumps({"gemm": name, "tokens": M, "gm": o, "ms": round(statistics.median(times[o]), 4),
                              "min_ms": round(min(times[o]), 4), "bitwise_equal_to_first": same[o]}), flush=True)
    h.gpp_order_config(prev)


if __name__ == "__main__":
    main()
