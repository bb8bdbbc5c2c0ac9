"""A/B of the ping-pong GEMM's two forms (gemm_pp.hip): one tile per workgroup vs the persistent kernel (one
workgroup per CU walking its tiles, the next tile's K-tile 0 prefetched across the seam), on the one-pass GEMMs
of a training step, interleaved over rounds on the same box, with hipBLASLt (torch.matmul) beside the plain ones.

    python benchmarks/gemm_persist_ab.py [--model gpt2|llama] [--tokens 131072] [--rounds 5]

Prints one JSON line per op: median ms per form, TF/s, and the persistent / one-tile ratio.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402

DIMS = {"gpt2": (768, 2048, 2304), "llama": (2048, 5632, 2560)}  # d, F, qkv width


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2", choices=list(DIMS))
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--head", action="store_true", help="the LM-head GEMMs (vocab 50432 padded) instead")
    a = ap.parse_args()
    if a.head:
        return head(a)
    h = ops()
    T = a.tokens
    d, F, Nq = DIMS[a.model]
    torch.manual_seed(0)
    bf = dict(device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, d, **bf)
    xf = torch.randn(T, F, **bf)
    dy = torch.randn(T, d, **bf)
    w13 = (0.05 * torch.randn(2 * F, d, device="cuda")).to(torch.bfloat16)
    w2 = (0.05 * torch.randn(d, F, device="cuda")).to(torch.bfloat16)
    wq = (0.05 * torch.randn(Nq, d, device="cuda")).to(torch.bfloat16)
    wo = (0.05 * torch.randn(d, d, device="cuda")).to(torch.bfloat16)
    gqkv = torch.randn(T, Nq, **bf)
    g13 = torch.randn(T, 2 * F, **bf)
    wq_t, w13_t = wq.t().contiguous(), w13.t().contiguous()
    cd = torch.empty(T, d, **bf)
    gu, _ = h.gemm_swiglu_fwd(x, w13)
    cq = torch.empty(T, Nq, **bf)
    co = torch.empty(T, d, **bf)
    cx = torch.empty(T, F, **bf)
    f = 2.0 * T
    ops_ = {
        "swiglu_fwd X.W13 (+gate)": (lambda: h.gemm_swiglu_fwd(x, w13), f * d * 2 * F, None),
        "swiglu_bwd dY.W2 (+gate bwd)": (lambda: h.gemm_swiglu_bwd(dy, w2, gu), f * d * F, None),
        "qkv fwd X.Wqkv^T": (lambda: h.gemm_pp(x, True, wq, True, cq, 0.0, 1), f * d * Nq,
                             lambda: torch.matmul(x, wq.t())),
        "o fwd X.Wo^T": (lambda: h.gemm_pp(x, True, wo, True, co, 0.0, 1), f * d * d, lambda: torch.matmul(x, wo.t())),
        "w2 fwd A.W2^T (K=F)": (lambda: h.gemm_pp(xf, True, w2, True, co, 0.0, 1), f * F * d,
                                lambda: torch.matmul(xf, w2.t())),
        "dX of w2: dY.W2 (B MN-major)": (lambda: h.gemm_pp(dy, True, w2, False, cx, 0.0, 1), f * d * F,
                                         lambda: torch.matmul(dy, w2)),
        # the input gradients the block backward runs (hipBLASLt in the TN layout through a transposed weight)
        "dX of qkv: dQKV.Wqkv (K=3d)": (lambda: h.gemm_pp(gqkv, True, wq_t, True, cd, 0.0, 1), f * Nq * d,
                                        lambda: torch.matmul(gqkv, wq_t.t())),
        "dX of qkv, B MN-major": (lambda: h.gemm_pp(gqkv, True, wq, False, cd, 0.0, 1), f * Nq * d, None),
        "dX of w13: dGU.W13 (K=2F)": (lambda: h.gemm_pp(g13, True, w13_t, True, cd, 0.0, 1), f * 2 * F * d,
                                      lambda: torch.matmul(g13, w13_t.t())),
        "dX of o: dY.Wo (K=d)": (lambda: h.gemm_pp(dy, True, wo.t().contiguous(), True, cd, 0.0, 1), f * d * d,
                                 lambda: torch.matmul(dy, wo)),
    }
    prev = h.gpp_persist_config(0)
    try:
        for name, (fn, flops, lib) in ops_.items():
            t = {0: [], 1: [], "lib": []}
            for mode in (0, 1):
                h.gpp_persist_config(mode)
                for _ in range(2):
                    fn()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for mode in (0, 1):
                    h.gpp_persist_config(mode)
                    t[mode].append(timeit(fn, a.iters))
                if lib is not None:
                    t["lib"].append(timeit(lib, a.iters))
            m0, m1 = statistics.median(t[0]), statistics.median(t[1])
            row = {"op": name, "model": a.model, "tokens": T, "tile_ms": round(m0, 4), "persist_ms": round(m1, 4),
                   "ratio": round(m1 / m0, 4), "tile_tflops": round(flops / m0 / 1e9, 1),
                   "persist_tflops": round(flops / m1 / 1e9, 1)}
            if t["lib"]:
                ml = statistics.median(t["lib"])
                row["hipblaslt_ms"] = round(ml, 4)
                row["hipblaslt_tflops"] = round(flops / ml / 1e9, 1)
            print(json.dumps(row), flush=True)
    finally:
        h.gpp_persist_config(prev)


def head(a):
    """LM head at GPT-2 width: logits = h . Wp^T (K = 768, 13.2 GB written) and dh = dlogits . Wp (K = 50432) on
    the persistent ping-pong kernel vs hipBLASLt (TN for dh, as ops/loss.py runs it)."""
    h_ = ops()
    T, d, V = a.tokens, 768, 50432
    bf = dict(device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, d, **bf)
    w = (0.05 * torch.randn(V, d, device="cuda")).to(torch.bfloat16)
    wt = w.t().contiguous()
    logits = torch.empty(T, V, **bf)
    dh = torch.empty(T, d, **bf)
    f = 2.0 * T * d * V
    arms = {
        "fwd pp": lambda: h_.gemm_pp(x, True, w, True, logits, 0.0, 1),
        "fwd hipBLASLt": lambda: torch.matmul(x, w.t(), out=logits),
        "dX pp (B K-major)": lambda: h_.gemm_pp(logits, True, wt, True, dh, 0.0, 1),
        "dX hipBLASLt TN": lambda: torch.matmul(logits, wt.t(), out=dh),
    }
    for fn in arms.values():
        fn()
    torch.cuda.synchronize()
    t = {k: [] for k in arms}
    for _ in range(a.rounds):
        for k, fn in arms.items():
            t[k].append(timeit(fn, 3))
    for k, v in t.items():
        m = statistics.median(v)
        print(json.dumps({"op": "lm head " + k, "tokens": T, "ms": round(m, 3), "tflops": round(f / m / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
