"""Weight-gradient GEMM dW += dY^T X at the GPT-2 B 128 shapes: the routes of ``ops/gemm.py`` (256-tile split-K
kernel, ping-pong kernel with both operands token-major) against the ping-pong kernel on a transposed copy of X
(``ppt``: X^T [K][T] makes B K-major, the MN x K layout; the transpose is timed with it).

    python benchmarks/dw_ppt.py [--model gpt2|llama]   (GPT-2 B 128: 131 072 tokens; Llama 1.1B: 65 536)

Prints one JSON line per shape: milliseconds (median of 5 rounds of 3) per route and the max relative difference
of each route's result from the first one's.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402
from bpe_transformer.ops.gemm import _run, choose_splits_pp  # noqa: E402


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2", choices=["gpt2", "llama"])
    a = ap.parse_args()
    h = ops()
    if a.model == "gpt2":
        T, shapes = 131072, [("qkv", 2304, 768), ("o", 768, 768), ("w13", 4096, 768), ("w2", 768, 2048),
                             ("head", 50432, 768)]
    else:
        T, shapes = 65536, [("qkv", 2560, 2048), ("o", 2048, 2048), ("w13", 11264, 2048), ("w2", 2048, 5632),
                            ("head", 32000, 2048)]
    for name, n, k in shapes:
        torch.manual_seed(0)
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16) * 0.01
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        res = {"shape": name, "N": n, "K": k, "T": T}
        outs = {}

        def ppt(g):
            xt = h.transpose_bf16(x)
            h.gemm_pp(dy, False, xt, True, g, 1.0, choose_splits_pp(n, k, T))

        routes = {"hip256": lambda g: _run("hip256", g, dy, x), "pp": lambda g: _run("pp", g, dy, x), "ppt": ppt}
        for r, fn in routes.items():
            g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
            try:
                fn(g)
            except RuntimeError as e:  # a route that does not take the shape
                res[f"{r}_ms"] = str(e).splitlines()[0][:80]
                continue
            torch.cuda.synchronize()
            outs[r] = g.float()
            res[f"{r}_ms"] = round(timed(lambda: fn(g)), 4)
        ref = next(iter(outs.values()))
        for r, o in outs.items():
            res[f"{r}_maxrel"] = float((o - ref).abs().max() / ref.abs().max())
        print(json.dumps(res), flush=True)
        del dy, x, outs


if __name__ == "__main__":
    main()
