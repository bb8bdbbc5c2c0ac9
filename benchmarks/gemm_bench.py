"""Microbenchmark: weight-gradient GEMMs (dW = dY^T X over all tokens), hipBLASLt vs the
hand-written split-K MFMA kernel (ops/csrc/gemm.hip), GPT-2-small shapes.  Random data,
median of interleaved timed rounds in one process (guide §5.4 rule 24)."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bpe_transformer import ops  # noqa: E402,F401  (loads the HIP library)
from bpe_transformer.ops.gemm import accumulate_weight_grad, choose_splits, matmul_nt  # noqa: E402


def bench(fn, iters=20):
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
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    T = a.tokens
    shapes = {"qkv": (2304, 768), "o": (768, 768), "w13": (4096, 768), "w2": (768, 2048)}
    out = {}
    for name, (n, k) in shapes.items():
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        g1 = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        g2 = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        t_blas, t_ours = [], []
        for _ in range(a.rounds):
            t_blas.append(bench(lambda: g1.addmm_(dy.t(), x)))
            t_ours.append(bench(lambda: accumulate_weight_grad(g2, dy, x)))
        fl = 2.0 * n * k * T
        mb, mo = statistics.median(t_blas), statistics.median(t_ours)
        out[name] = {"shape": [n, k, T], "splits": choose_splits(n, k, T), "hipblaslt_ms": round(mb, 4),
                     "ours_ms": round(mo, 4), "hipblaslt_tflops": round(fl / mb / 1e9, 1),
                     "ours_tflops": round(fl / mo / 1e9, 1), "speedup": round(mb / mo, 3)}
        print(json.dumps({name: out[name]}), flush=True)
    # forward-shaped products Y = X W^T (both operands K-major): hipBLASLt vs the same kernel
    for name, (n, k) in shapes.items():
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(T, n, device="cuda", dtype=torch.bfloat16)
        tb, to = [], []
        for _ in range(a.rounds):
            tb.append(bench(lambda: torch.matmul(x, w.t(), out=y)))
            to.append(bench(lambda: matmul_nt(x, w, out=y)))
        fl = 2.0 * n * k * T
        mb, mo = statistics.median(tb), statistics.median(to)
        print(json.dumps({"fwd_" + name: {"hipblaslt_tflops": round(fl / mb / 1e9, 1),
                                          "ours_tflops": round(fl / mo / 1e9, 1), "speedup": round(mb / mo, 3)}}),
              flush=True)


if __name__ == "__main__":
    main()
