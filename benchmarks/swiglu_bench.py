"""SwiGLU kernels at GPT-2-small training shapes (bf16): the gate forward, the X.W13 GEMM with the gate in its
epilogue and the unfused pair it replaces (hipBLASLt X.W13^T + swiglu_fwd), the standalone backward, the dY.W2
GEMM with the SwiGLU backward in its epilogue, and the unfused pair it replaces (hipBLASLt dY.W2 + swiglu_bwd).

    python benchmarks/swiglu_bench.py [--tokens 131072] [--dim 768] [--ff 2048]

Prints one JSON line per op: ms, effective TB/s (bytes the op must move) and, for the GEMMs, TF/s.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--ff", type=int, default=2048)
    a = ap.parse_args()
    M, d, F = a.tokens, a.dim, a.ff
    h = ops()
    torch.manual_seed(0)
    gu = torch.randn(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    w2 = (0.05 * torch.randn(d, F, device="cuda")).to(torch.bfloat16)
    da = torch.randn(M, F, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    w13 = (0.05 * torch.randn(2 * F, d, device="cuda")).to(torch.bfloat16)
    gemm_flops = 2.0 * M * d * F
    rows = {
        "swiglu_fwd": (lambda: h.swiglu_fwd(gu), 3 * M * F * 2, 0.0),
        "gemm_swiglu_fwd(fused)": (lambda: h.gemm_swiglu_fwd(x, w13), 3 * M * F * 2, 2 * gemm_flops),
        "X@W13 (hipBLASLt)": (lambda: torch.matmul(x, w13.t()), 2 * M * F * 2, 2 * gemm_flops),
        "X@W13 + swiglu_fwd (unfused)": (lambda: h.swiglu_fwd(torch.matmul(x, w13.t())), 5 * M * F * 2,
                                         2 * gemm_flops),
        "swiglu_bwd": (lambda: h.swiglu_bwd(da, gu), 5 * M * F * 2, 0.0),
        "gemm_swiglu_bwd(fused)": (lambda: h.gemm_swiglu_bwd(dy, w2, gu), 4 * M * F * 2, gemm_flops),
        "dY@W2 (hipBLASLt)": (lambda: torch.matmul(dy, w2), M * F * 2, gemm_flops),
        "dY@W2 + swiglu_bwd (unfused)": (lambda: h.swiglu_bwd(torch.matmul(dy, w2), gu), 6 * M * F * 2, gemm_flops),
    }
    for name, (fn, nbytes, flops) in rows.items():
        ms = timeit(fn)
        r = {"op": name, "shape": [M, d, F], "ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 2)}
        if flops:
            r["TFps"] = round(flops / ms / 1e9, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
