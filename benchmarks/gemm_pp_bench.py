"""Ping-pong GEMM (csrc/gemm_pp.hip) vs hipBLASLt on the training-step shapes.

For every projection of the GPT-2-small (and Llama-1.1B) step: forward Y = X W^T, input gradient dX = dY W,
weight gradient dW = dY^T X, each timed on our kernel and on torch.matmul (hipBLASLt), after a numerics check
against the library result.  Prints one JSON line per shape.

    python benchmarks/gemm_pp_bench.py [--model gpt2|llama|both] [--tokens 65536]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpe_transformer.ops._ext import ops  # noqa: E402

SHAPES = {
    "gpt2": {"qkv": (2304, 768), "o": (768, 768), "w13": (4096, 768), "w2": (768, 2048), "head": (50432, 768)},
    "llama": {"qkv": (2560, 2048), "o": (2048, 2048), "w13": (11264, 2048), "w2": (2048, 5632),
              "head": (32000, 2048)},
}


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def rel_err(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def choose_splits(m, n, r, cus=256):
    tiles = (m // 256) * (n // 256)
    nk = r // 64
    best, best_cost = 1, None
    for s in range(1, 65):
        if nk // s < 4:
            break
        waves = -(-tiles * s // cus)
        cost = waves * (-(-nk // s)) + (0.15 * s * m * n / 65536 if s > 1 else 0.0) / 16
        if best_cost is None or cost < best_cost * 0.97:
            best, best_cost = s, cost
    return best


def run_quick(name, n, k, t, dev):
    """Time only the ping-pong kernel (no checks): for A/B builds (BPE_HIP_VARIANT) and diagnostics."""
    x = torch.randn(t, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(t, n, device=dev, dtype=torch.bfloat16)
    y = torch.empty(t, n, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(t, k, device=dev, dtype=torch.bfloat16)
    g = torch.zeros(n, k, device=dev, dtype=torch.bfloat16)
    s = choose_splits(n, k, t)
    fl = 2.0 * t * n * k
    res = {"name": name}
    for kind, fn in (("fwd", lambda: ops().gemm_pp(x, True, w, True, y, 0.0, 1)),
                     ("dX", lambda: ops().gemm_pp(dy, True, w, False, dx, 0.0, 1)),
                     ("dW", lambda: ops().gemm_pp(dy, False, x, False, g, 1.0, s))):
        ms = bench(fn, 20)
        res[f"{kind}_tf"] = round(fl / ms * 1e-9, 1)
    return res


def run_shape(name, n, k, t, dev):
    torch.manual_seed(0)
    x = torch.randn(t, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.05
    dy = torch.randn(t, n, device=dev, dtype=torch.bfloat16)
    res = {"name": name, "N": n, "K": k, "T": t}
    # forward
    y_ref = x @ w.t()
    y = torch.empty_like(y_ref)
    ops().gemm_pp(x, True, w, True, y, 0.0, 1)
    res["fwd_err"] = rel_err(y, y_ref)
    fl = 2.0 * t * n * k
    res["fwd_blas_ms"] = bench(lambda: torch.matmul(x, w.t(), out=y_ref))
    res["fwd_pp_ms"] = bench(lambda: ops().gemm_pp(x, True, w, True, y, 0.0, 1))
    # input gradient
    dx_ref = dy @ w
    dx = torch.empty_like(dx_ref)
    ops().gemm_pp(dy, True, w, False, dx, 0.0, 1)
    res["dX_err"] = rel_err(dx, dx_ref)
    res["dX_blas_ms"] = bench(lambda: torch.matmul(dy, w, out=dx_ref))
    res["dX_pp_ms"] = bench(lambda: ops().gemm_pp(dy, True, w, False, dx, 0.0, 1))
    # weight gradient (accumulate, as in training)
    s = choose_splits(n, k, t)
    g_ref = dy.t() @ x
    g = torch.zeros_like(g_ref)
    ops().gemm_pp(dy, False, x, False, g, 1.0, s)
    res["dW_err"] = rel_err(g, g_ref)
    res["dW_splits"] = s
    res["dW_blas_ms"] = bench(lambda: g_ref.addmm_(dy.t(), x))
    res["dW_pp_ms"] = bench(lambda: ops().gemm_pp(dy, False, x, False, g, 1.0, s))
    if n % 256 == 0 and k % 256 == 0:
        res["dW_g256_ms"] = bench(lambda: ops().gemm(dy, False, x, False, g, 1.0, s, 256))
    for kind in ("fwd", "dX", "dW"):
        for impl in ("blas", "pp", "g256"):
            key = f"{kind}_{impl}_ms"
            if key in res:
                res[f"{kind}_{impl}_tf"] = round(fl / res[key] * 1e-9, 1)
                res[key] = round(res[key], 4)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--tokens", type=int, default=None)
    ap.add_argument("--only", default=None)
    ap.add_argument("--quick", action="store_true", help="time the ping-pong kernel only")
    a = ap.parse_args()
    dev = torch.device("cuda")
    models = ["gpt2", "llama"] if a.model == "both" else [a.model]
    for m in models:
        t = a.tokens or (65536 if m == "gpt2" else 16384)
        for name, (n, k) in SHAPES[m].items():
            if a.only and name not in a.only.split(","):
                continue
            fn = run_quick if a.quick else run_shape
            print(json.dumps({"model": m, "variant": os.environ.get("BPE_HIP_VARIANT"),
                              "diag": os.environ.get("BPE_GPP_DIAG"), **fn(name, n, k, t, dev)}), flush=True)


if __name__ == "__main__":
    main()
