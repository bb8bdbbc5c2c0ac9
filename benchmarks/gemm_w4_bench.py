"""The 4-wave persistent GEMM (gemm_w4.hip; w4 = the ring form, w4s = the 2-stage form, w4g = the register-staged ring) against the persistent ping-pong kernel (gemm_pp.hip) and hipBLASLt
(torch.matmul) on the one-pass GEMMs of a training step, interleaved over rounds in one process (guide §5.4 rule 24).

    python benchmarks/gemm_w4_bench.py [--model gpt2|llama] [--tokens 131072] [--rounds 5]

Prints one JSON line per op: median ms and TF/s per arm.
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
    ap.add_argument("--square", type=int, default=0, help="also an N x N x N GEMM of this size")
    a = ap.parse_args()
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
    wq_t, w13_t, wo_t = wq.t().contiguous(), w13.t().contiguous(), wo.t().contiguous()
    f = 2.0 * T
    # (name, A, a_kmajor, B, b_kmajor, out, flops)
    cases = [
        ("qkv fwd X.Wqkv^T", x, True, wq, True, torch.empty(T, Nq, **bf), f * d * Nq),
        ("o fwd X.Wo^T", x, True, wo, True, torch.empty(T, d, **bf), f * d * d),
        ("w13 fwd X.W13^T", x, True, w13, True, torch.empty(T, 2 * F, **bf), f * d * 2 * F),
        ("w2 fwd A.W2^T (K=F)", xf, True, w2, True, torch.empty(T, d, **bf), f * F * d),
        ("dX of qkv (TN, K=3d)", gqkv, True, wq_t, True, torch.empty(T, d, **bf), f * Nq * d),
        ("dX of w13 (TN, K=2F)", g13, True, w13_t, True, torch.empty(T, d, **bf), f * 2 * F * d),
        ("dX of o (TN, K=d)", dy, True, wo_t, True, torch.empty(T, d, **bf), f * d * d),
        ("dX of w2: dY.W2 (B MN-major)", dy, True, w2, False, torch.empty(T, F, **bf), f * d * F),
        ("dX of qkv, B MN-major", gqkv, True, wq, False, torch.empty(T, d, **bf), f * Nq * d),
    ]
    if a.square:
        n = a.square
        sa = torch.randn(n, n, **bf)
        sb = torch.randn(n, n, **bf)
        cases.append((f"square {n}", sa, True, sb, True, torch.empty(n, n, **bf), 2.0 * n ** 3))
    for name, A, ak, B, bk, out, flops in cases:
        def w4(ring):
            def f():
                prev = h.gw4_ring_config(ring)
                h.gemm_w4(A, ak, B, bk, out, 0.0)
                h.gw4_ring_config(prev)
            return f

        arms = {
            "w4": w4(1),
            "w4s": w4(0),
            "w4g": w4(2),
            "pp": lambda: h.gemm_pp(A, ak, B, bk, out, 0.0, 1),
            "lib": (lambda: torch.matmul(A, B.t(), out=out)) if bk else (lambda: torch.matmul(A, B, out=out)),
        }
        if not ak:
            arms["lib"] = lambda: torch.matmul(A.t(), B.t() if bk else B, out=out)
        ref = None
        for k, fn in arms.items():
            fn()
            if ref is None:
                ref = out.float().clone()
            else:
                err = float((out.float() - ref).abs().max() / ref.abs().max())
                assert err < 2e-2, (name, k, err)
        torch.cuda.synchronize()
        t = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                t[k].append(timeit(fn, a.iters))
        row = {"op": name, "model": a.model, "tokens": T}
        for k, v in t.items():
            m = statistics.median(v)
            row[f"{k}_ms"] = round(m, 4)
            row[f"{k}_tflops"] = round(flops / m / 1e9, 1)
        row["w4_vs_w4s"] = round(row["w4s_ms"] / row["w4_ms"], 3)
        row["w4g_vs_pp"] = round(row["pp_ms"] / row["w4g_ms"], 3)
        row["w4_vs_pp"] = round(row["pp_ms"] / row["w4_ms"], 3)
        row["w4_vs_lib"] = round(row["lib_ms"] / row["w4_ms"], 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
