"""Main-loop rate of the ping-pong GEMM per operand layout: C = A . B^T over a long reduction, one split, with each
operand K-major (reduction index contiguous) or MN-major, at shapes large enough that the loop dominates.

    python benchmarks/gemm_pp_layouts.py

Prints one JSON line per (shape, layout): median ms and TF/s (the weight gradient dW = dY^T X is the MN x MN
layout; the forward K x K; the input gradient K x MN).
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def timeit(fn, iters=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    h = ops()
    for M, N, K in [(4096, 4096, 16384), (11264, 2048, 32768), (2048, 2048, 65536)]:
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        At, Bt = A.t().contiguous(), B.t().contiguous()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        arms = {"KxK": (A, True, B, True), "KxMN": (A, True, Bt, False), "MNxK": (At, False, B, True),
                "MNxMN": (At, False, Bt, False)}
        t = {k: [] for k in arms}
        for _ in range(3):
            for k, (a, ak, b, bk) in arms.items():
                t[k].append(timeit(lambda: h.gemm_pp(a, ak, b, bk, C, 0.0, 1)))
        t["hipblaslt KxK"] = [timeit(lambda: torch.matmul(A, B.t(), out=C)) for _ in range(3)]
        for k, v in t.items():
            m = statistics.median(v)
            print(json.dumps({"MNK": [M, N, K], "layout": k, "ms": round(m, 4), "tflops": round(fl / m / 1e9, 1)}),
                  flush=True)
        del A, B, At, Bt, C


if __name__ == "__main__":
    main()
