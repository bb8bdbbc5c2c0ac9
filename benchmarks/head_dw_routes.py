"""LM-head weight gradient dW += dlogits^T h (50432 x 768 over 131072 tokens at GPT-2 B 128) on each route of
ops/gemm.py: the ping-pong split-K kernel ("pp"), the 256-tile split-K kernel ("hip256") and hipBLASLt
("blas", addmm_; tuned when run with PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1).  Random data,
median of interleaved rounds, one JSON line.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def bench(fn, iters=5):
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
    from bpe_transformer.ops.gemm import _candidates, _run

    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--n", type=int, default=50432)
    ap.add_argument("--k", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    T, N, K = a.tokens, a.n, a.k
    bf = torch.bfloat16
    dl = torch.randn(T, N, device="cuda", dtype=bf)
    h = torch.randn(T, K, device="cuda", dtype=bf)
    g = torch.zeros(N, K, device="cuda", dtype=bf)
    cands = _candidates(N, K, T)
    r = {c: [] for c in cands}
    for _ in range(a.rounds):
        for c in cands:
            r[c].append(bench(lambda: _run(c, g, dl, h)))
    fl = 2.0 * T * N * K
    row = {"shape": [N, K, T]}
    for c, v in r.items():
        m = statistics.median(v)
        row[c + "_ms"] = round(m, 3)
        row[c + "_tflops"] = round(fl / m / 1e9, 1)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
