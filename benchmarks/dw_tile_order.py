"""Weight-gradient GEMMs (split-K ping-pong kernel, fp32 slab + ordered reduce) under the tile orders of
``gpp_order_config`` (gemm_pp.hip tile_rc, applied inside each split's tile grid when set explicitly).

    python benchmarks/dw_tile_order.py [--tokens 65536] [--shapes 11264x2048:ppt,2560x2048:pp,2048x2048:pp]

One JSON line per (shape, route, order): median ms of interleaved repetitions and TF/s.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402
from bpe_transformer.ops.gemm import choose_splits_pp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--shapes", default="11264x2048:ppt,2560x2048:pp,2048x2048:pp")
    ap.add_argument("--orders", default="0,2,4,8")
    a = ap.parse_args()
    h = ops()
    T = a.tokens
    orders = [int(x) for x in a.orders.split(",")]
    prev = h.gpp_order_config(-1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for spec in a.shapes.split(","):
        nk, route = spec.split(":")
        n, k = (int(v) for v in nk.split("x"))
        torch.manual_seed(0)
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        xt = h.transpose_bf16(x)
        g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        s = choose_splits_pp(n, k, T)
        fn = (lambda: h.gemm_pp(dy, False, xt, True, g, 0.0, s)) if route == "ppt" else \
            (lambda: h.gemm_pp(dy, False, x, False, g, 0.0, s))
        times = {o: [] for o in orders}
        for _ in range(5):
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
            ms = statistics.median(times[o])
            print(json.dumps({"N": n, "K": k, "T": T, "route": route, "splits": s, "gm": o, "ms": round(ms, 4),
                              "tflops": round(2 * n * k * T / ms / 1e9, 1)}), flush=True)
        del dy, x, xt, g
    h.gpp_order_config(prev)


if __name__ == "__main__":
    main()
