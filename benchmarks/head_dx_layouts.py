"""LM-head input gradient dh = dlogits @ W in both hipBLASLt layouts, each with its TunableOp-tuned solution.

  NN : torch.matmul(dlogits, W)            W [V][d] row-major (reduction index V strided by d)
  TN : torch.matmul(dlogits, Wt.t())       Wt = W^T materialised [d][V] (both operands V-contiguous)

Run with PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=<csv>: the first call
of each layout tunes it (the chosen solutions land in the csv), then both are timed interleaved on random data.
"""
import argparse
import json
import statistics

import torch


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--vocab", type=int, default=50432)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    T, V, d = a.tokens, a.vocab, a.dim
    bf = torch.bfloat16
    dl = torch.randn(T, V, device="cuda", dtype=bf)
    w = torch.randn(V, d, device="cuda", dtype=bf) * 0.02
    wt = w.t().contiguous()
    out = torch.empty(T, d, device="cuda", dtype=bf)
    r = {"NN": [], "TN": [], "transpose": []}
    for _ in range(a.rounds):
        r["NN"].append(bench(lambda: torch.matmul(dl, w, out=out)))
        r["TN"].append(bench(lambda: torch.matmul(dl, wt.t(), out=out)))
        r["transpose"].append(bench(lambda: wt.copy_(w.t())))
    fl = 2.0 * T * V * d
    row = {"shape": [T, V, d]}
    for k, v in r.items():
        m = statistics.median(v)
        row[k + "_ms"] = round(m, 4)
        if k != "transpose":
            row[k + "_tflops"] = round(fl / m / 1e9, 1)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
