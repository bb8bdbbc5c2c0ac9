"""Probe: weight-gradient GEMM dW = dY^T X with token-major operands (MN-major, ds_read_b64_tr_b16 fragments) vs
the same product from pre-transposed operands (K-major, ds_read_b128 fragments), on the ping-pong kernel, plus the
8192^3 square ceiling of kernel and library.  Prints one JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpe_transformer.ops._ext import ops  # noqa: E402
from bpe_transformer.ops.gemm import choose_splits_pp  # noqa: E402


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


def main():
    dev = torch.device("cuda")
    T = int(os.environ.get("T", "131072"))
    for name, (n, k) in {"qkv": (2304, 768), "o": (768, 768), "w13": (4096, 768), "w2": (768, 2048)}.items():
        x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
        xt = x.t().contiguous()
        dyt = dy.t().contiguous()
        g = torch.zeros(n, k, device=dev, dtype=torch.bfloat16)
        s = choose_splits_pp(n, k, T)
        fl = 2.0 * T * n * k
        r = {"name": name, "n": n, "k": k, "T": T, "splits": s}
        r["mn_major_tf"] = round(fl / bench(lambda: ops().gemm_pp(dy, False, x, False, g, 1.0, s)) * 1e-9, 1)
        r["k_major_tf"] = round(fl / bench(lambda: ops().gemm_pp(dyt, True, xt, True, g, 1.0, s)) * 1e-9, 1)
        r["blas_tf"] = round(fl / bench(lambda: g.addmm_(dy.t(), x)) * 1e-9, 1)
        r["transpose_ms"] = round(bench(lambda: xt.copy_(x.t())), 4)
        print(json.dumps(r), flush=True)
    for m in (4096, 8192):
        a = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
        b = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
        c = torch.empty(m, m, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * m ** 3
        print(json.dumps({"square": m, "pp_nt_tf": round(fl / bench(lambda: ops().gemm_pp(a, True, b, True, c, 0.0, 1)) * 1e-9, 1),
                          "blas_nt_tf": round(fl / bench(lambda: torch.matmul(a, b.t(), out=c)) * 1e-9, 1)}), flush=True)


if __name__ == "__main__":
    main()
