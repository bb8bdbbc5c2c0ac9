"""Microbenchmark: every projection GEMM of one training step (forward, input-gradient, weight-gradient)
at the model's real shapes, in each operand layout the library / our kernel can run it in.

  fwd : Y  = X  @ W^T        X [T,K], W [N,K]            (both operands K-contiguous)
  fwdN: Y  = X  @ Wt         Wt = W^T materialised [K,N] (the copy the TN input gradient makes)
  dX  : dX = dY @ W          dY [T,N], W [N,K]           (B is N-contiguous: the "NN" layout)
  dXt : dX = dY @ (W^T)^T    with W^T materialised once  (back to the K-contiguous layout; the
                                                          transpose copy is timed separately)
  dW  : dW += dY^T @ X       hipBLASLt addmm_ vs ops.gemm split-K MFMA kernel

Random data, median of interleaved rounds in one process.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bpe_transformer import ops  # noqa: E402,F401
from bpe_transformer.models import get_preset  # noqa: E402
from bpe_transformer.ops._ext import ops as hip  # noqa: E402
from bpe_transformer.ops.gemm import choose_splits, choose_splits_256, use_tile256  # noqa: E402


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
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    cfg = get_preset(a.model)
    d, f, hd = cfg.d_model, cfg.d_ff, cfg.d_model // cfg.num_heads
    kv = (cfg.num_kv_heads or cfg.num_heads) * hd
    shapes = {"qkv": (d + 2 * kv, d), "o": (d, d), "w13": (2 * f, d), "w2": (d, f), "lm_head": (cfg.vocab_size, d)}
    T = a.tokens
    bf = torch.bfloat16
    tot = {"fwd": 0.0, "dX": 0.0, "dXt": 0.0, "dW_blas": 0.0, "dW_best": 0.0}
    for name, (n, k) in shapes.items():
        x = torch.randn(T, k, device="cuda", dtype=bf)
        w = torch.randn(n, k, device="cuda", dtype=bf) * 0.02
        dy = torch.randn(T, n, device="cuda", dtype=bf)
        y = torch.empty(T, n, device="cuda", dtype=bf)
        dx = torch.empty(T, k, device="cuda", dtype=bf)
        wt = w.t().contiguous()
        g = torch.zeros(n, k, device="cuda", dtype=bf)
        r = {k_: [] for k_ in ("fwd", "fwdN", "dX", "dXt", "tr", "dW_blas", "dW_ours", "dW_256")}
        ours_ok = n % 128 == 0 and k % 128 == 0
        s128 = choose_splits(n, k, T)
        s256 = choose_splits_256(n, k, T) if use_tile256(n, k, T) else None
        for _ in range(a.rounds):
            r["fwd"].append(bench(lambda: torch.matmul(x, w.t(), out=y)))
            r["fwdN"].append(bench(lambda: torch.matmul(x, wt, out=y)))
            r["dX"].append(bench(lambda: torch.matmul(dy, w, out=dx)))
            r["dXt"].append(bench(lambda: torch.matmul(dy, wt.t(), out=dx)))
            r["tr"].append(bench(lambda: wt.copy_(w.t())))
            r["dW_blas"].append(bench(lambda: g.addmm_(dy.t(), x)))
            if ours_ok:
                r["dW_ours"].append(bench(lambda: hip().gemm(dy, False, x, False, g, 1.0, s128, 128)))
            if s256:
                r["dW_256"].append(bench(lambda: hip().gemm(dy, False, x, False, g, 1.0, s256, 256)))
        med = {k_: statistics.median(v) for k_, v in r.items() if v}
        fl = 2.0 * n * k * T
        row = {"shape": [n, k, T], "splits128": s128, "splits256": s256}
        for k_, v in med.items():
            row[k_ + "_ms"] = round(v, 4)
            if k_ != "tr":
                row[k_ + "_tflops"] = round(fl / v / 1e9, 1)
        print(json.dumps({name: row}), flush=True)
        if s256:  # calibrate the split model
            sweep = {}
            for sp in (1, 2, 4, 8, 16, 32):
                if (T // 64) % sp == 0 and T // 64 // sp >= 4:
                    sweep[sp] = round(bench(lambda: hip().gemm(dy, False, x, False, g, 1.0, sp, 256)), 4)
            print(json.dumps({name + "_sweep256_ms": sweep}), flush=True)
        if name == "lm_head":
            continue
        tot["fwd"] += med["fwd"]
        tot["dX"] += med["dX"]
        tot["dXt"] += med["dXt"] + med["tr"]
        tot["dW_blas"] += med["dW_blas"]
        tot["dW_best"] += min(med["dW_blas"], med.get("dW_ours", 1e9), med.get("dW_256", 1e9))
    print(json.dumps({"per_layer_ms": {k_: round(v, 4) for k_, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
