"""Split-K sweep of the ping-pong kernel on the weight-gradient shapes routed to it (``pp``: both operands
token-major; ``ppt``: X transposed first, not timed here), against the split count ``ops.gemm.choose_splits_pp``
picks.

    python benchmarks/dw_splits.py

Prints one JSON line per shape: {splits: ms} (median of 5 rounds of 3) and the model's choice.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402
from bpe_transformer.ops.gemm import choose_splits_pp  # noqa: E402

SHAPES = [("gpt2 qkv", "pp", 2304, 768, 131072), ("gpt2 head", "ppt", 50432, 768, 131072),
          ("llama qkv", "pp", 2560, 2048, 65536), ("llama o", "pp", 2048, 2048, 65536),
          ("llama w13", "ppt", 11264, 2048, 65536), ("llama head", "ppt", 32000, 2048, 65536)]


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    out = []
    for _ in range(5):
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        out.append(ev[0].elapsed_time(ev[1]) / reps)
    return statistics.median(out)


def main():
    h = ops()
    for name, route, n, k, t in SHAPES:
        torch.manual_seed(0)
        dy = torch.randn(t, n, device="cuda", dtype=torch.bfloat16) * 0.01
        x = torch.randn(t, k, device="cuda", dtype=torch.bfloat16)
        b, bk = (h.transpose_bf16(x), True) if route == "ppt" else (x, False)
        g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        tiles = (n // 256) * (k // 256)
        res = {"shape": name, "route": route, "N": n, "K": k, "T": t, "tiles": tiles,
               "model_splits": choose_splits_pp(n, k, t), "ms": {}}
        for s in (1, 2, 3, 4, 5, 6, 8, 9, 10, 12, 16, 19, 24, 28, 32):
            if tiles * s > 8192 or t // 64 < 4 * s:
                continue
            res["ms"][s] = round(timed(lambda: h.gemm_pp(dy, False, b, bk, g, 1.0, s)), 4)
        print(json.dumps(res), flush=True)
        del dy, x, b, g


if __name__ == "__main__":
    main()
