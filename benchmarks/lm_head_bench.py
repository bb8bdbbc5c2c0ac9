"""Microbenchmark: the GPT-2 LM-head GEMMs at the raw vocab (50257) vs padded vocabs.

logits = h W^T (fwd), dh = dlogits W (dX), dW += dlogits^T h (dW), with M = 65536 tokens, d = 768.
An odd vocab makes the logits' row stride odd (100514 bytes), which rules out the libraries' vectorised
row accesses; padding W with zero rows to a multiple of 64/256 keeps every stride 128-byte aligned.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bpe_transformer import ops  # noqa: E402,F401
from bpe_transformer.ops.gemm import _run, use_tile256  # noqa: E402


def bench(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--vocabs", default="50257,50304,50432")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    M, d = a.tokens, a.d
    h = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    for V in [int(v) for v in a.vocabs.split(",")]:
        w = torch.randn(V, d, device="cuda", dtype=torch.bfloat16) * 0.02
        logits = torch.empty(M, V, device="cuda", dtype=torch.bfloat16)
        dh = torch.empty(M, d, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(V, d, device="cuda", dtype=torch.bfloat16)
        res = {"fwd": [], "dX": [], "dW_blas": [], "dW_hip": []}
        for _ in range(a.rounds):
            res["fwd"].append(bench(lambda: torch.matmul(h, w.t(), out=logits)))
            res["dX"].append(bench(lambda: torch.matmul(logits, w, out=dh)))
            res["dW_blas"].append(bench(lambda: g.addmm_(logits.t(), h)))
            if use_tile256(V, d, M):
                res["dW_hip"].append(bench(lambda: _run("hip256", g, logits, h)))
        fl = 2.0 * M * V * d
        out = {"vocab": V}
        for k, v in res.items():
            if v:
                ms = statistics.median(v)
                out[k + "_ms"] = round(ms, 3)
                out[k + "_tflops"] = round(fl / ms / 1e9, 1)
        print(json.dumps(out), flush=True)
        del w, logits, g, dh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
