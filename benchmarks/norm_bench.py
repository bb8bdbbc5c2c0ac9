"""Memory-bound block kernels at training shapes (bf16): RMSNorm forward, residual-add forward, backward with
the fused residual gradient, SwiGLU forward.  Prints ms and effective TB/s (bytes each kernel must move) per op.

    python benchmarks/norm_bench.py [--rows 65536] [--dim 768]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
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
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=768)
    a = ap.parse_args()
    M, N = a.rows, a.dim
    h = ops()
    x = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    d = torch.randn_like(x)
    w = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn_like(x)
    dres = torch.randn_like(x)
    _, rstd = h.rmsnorm_fwd(x, w, 1e-5)
    B = M * N * 2
    rows = {
        "rmsnorm_fwd": (lambda: h.rmsnorm_fwd(x, w, 1e-5), 2 * B),
        "add_rmsnorm_fwd": (lambda: h.add_rmsnorm_fwd(x, d, w, 1e-5), 4 * B),
        "rmsnorm_bwd+dres": (lambda: h.rmsnorm_bwd(dy, x, w, rstd, dres), 4 * B),
    }
    F = 4 * N if N < 2048 else 2816
    gu = torch.randn(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    rows["swiglu_fwd"] = (lambda: h.swiglu_fwd(gu), 3 * M * F * 2)
    for name, (fn, nbytes) in rows.items():
        ms = timeit(fn)
        print(json.dumps({"op": name, "shape": [M, N], "ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
