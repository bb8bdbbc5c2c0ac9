"""LM-head GEMMs of one training step in every operand layout hipBLASLt / our kernels can run them in, each
library layout with its TunableOp-tuned solution (run with PYTORCH_TUNABLEOP_ENABLED=1
PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=<csv>: the first call of each layout tunes it).

  fwd  TN : logits = h @ W^T                  (both operands d-contiguous; the default)
  fwd  NN : logits = h @ Wt                   Wt = W^T materialised [d][V] (the copy the TN dX already makes)
  dX   NN : dh = dlogits @ W
  dX   TN : dh = dlogits @ Wt^T
  dW   pp : dW += dlogits^T hs                ping-pong MFMA kernel, split-K (ops.gemm route "pp")
  dW   NT : dW = dlogits^T @ hs               hipBLASLt
  dWt  TN : dW^T = hs^T @ dlogits  (+ transpose back)

Random N(0,1) data, median of interleaved rounds.  One JSON line.
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
    from bpe_transformer.ops._ext import ops as hip

    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--vocab", type=int, default=50432)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    T, V, d = a.tokens, a.vocab, a.dim
    bf = torch.bfloat16
    h = torch.randn(T, d, device="cuda", dtype=bf)
    dl = torch.randn(T, V, device="cuda", dtype=bf)
    w = torch.randn(V, d, device="cuda", dtype=bf) * 0.02
    wt = hip().transpose_bf16(w)
    logits = torch.empty(T, V, device="cuda", dtype=bf)
    dh = torch.empty(T, d, device="cuda", dtype=bf)
    dw = torch.zeros(V, d, device="cuda", dtype=bf)
    dwt = torch.empty(d, V, device="cuda", dtype=bf)
    from bpe_transformer.ops.gemm import accumulate_weight_grad

    r = {k: [] for k in ("fwd_TN", "fwd_NN", "dX_NN", "dX_TN", "dW_pp", "dW_NT", "dWt_TN", "transpose")}
    for _ in range(a.rounds):
        r["fwd_TN"].append(bench(lambda: torch.matmul(h, w.t(), out=logits)))
        r["fwd_NN"].append(bench(lambda: torch.matmul(h, wt, out=logits)))
        r["dX_NN"].append(bench(lambda: torch.matmul(dl, w, out=dh)))
        r["dX_TN"].append(bench(lambda: torch.matmul(dl, wt.t(), out=dh)))
        r["dW_pp"].append(bench(lambda: accumulate_weight_grad(dw, dl, h)))
        r["dW_NT"].append(bench(lambda: torch.matmul(dl.t(), h, out=dw)))
        r["dWt_TN"].append(bench(lambda: torch.matmul(h.t(), dl, out=dwt)))
        r["transpose"].append(bench(lambda: hip().transpose_bf16(w)))
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
