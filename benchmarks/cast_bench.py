"""fp8 cast kernels at the fp8 Llama config's tensor shapes (65 536 tokens): the two-layout cast (cast_fp8_t), the
plain row-major cast (cast_fp8) and a bf16 copy for the HBM reference, in effective TB/s (bytes read + written).

    python benchmarks/cast_bench.py
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def timeit(fn, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    h = ops()
    for T, N in [(65536, 2048), (65536, 2560), (65536, 11264), (2560, 2048)]:
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        s = torch.ones(1, device="cuda")
        am = torch.zeros(1, dtype=torch.int32, device="cuda")
        o8 = torch.empty(T, N, dtype=torch.float8_e5m2, device="cuda")
        o8t = torch.empty(N, T, dtype=torch.float8_e5m2, device="cuda")
        y = torch.empty_like(x)
        arms = {"cast_t": (lambda: h.cast_fp8_t(x, s, o8, o8t, am), 4),
                "cast": (lambda: h.cast_fp8(x, s, o8, am), 3),
                "bf16_copy": (lambda: y.copy_(x), 4)}
        t = {k: [] for k in arms}
        for _ in range(3):
            for k, (fn, _) in arms.items():
                t[k].append(timeit(fn))
        for k, (_, bpe) in arms.items():
            m = statistics.median(t[k])
            print(json.dumps({"shape": [T, N], "op": k, "us": round(m * 1e3, 1),
                              "TBps": round(T * N * bpe / m / 1e9, 2)}), flush=True)
    # the SwiGLU + two-layout casts at Llama width (gu = [g | u], F = 5632): forward reads gu and writes a8 / a8t
    # (2F + 2F bytes per token... 4F + 2F), backward also reads dA and writes both layouts of [dg | du]
    T, F = 65536, 5632
    gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    da = torch.randn(T, F, device="cuda", dtype=torch.bfloat16)
    s = torch.ones(1, device="cuda")
    am = torch.zeros(1, dtype=torch.int32, device="cuda")
    a8 = torch.empty(T, F, dtype=torch.float8_e4m3fn, device="cuda")
    a8t = torch.empty(F, T, dtype=torch.float8_e4m3fn, device="cuda")
    g8 = torch.empty(T, 2 * F, dtype=torch.float8_e5m2, device="cuda")
    g8t = torch.empty(2 * F, T, dtype=torch.float8_e5m2, device="cuda")
    arms = {"swiglu_cast_fwd": (lambda: h.swiglu_cast_fp8_t(gu, None, s, a8, a8t, am), T * F * (4 + 2)),
            "swiglu_cast_bwd": (lambda: h.swiglu_cast_fp8_t(gu, da, s, g8, g8t, am), T * F * (4 + 2 + 4))}
    # residual add + RMSNorm with the e4m3 output, then its fp8 transpose (add_rmsnorm_cast_fp8_t), at d 2048
    N = 2048
    xx = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    dd = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    ww = torch.rand(N, device="cuda", dtype=torch.bfloat16) + 0.5
    y8 = torch.empty(T, N, dtype=torch.float8_e4m3fn, device="cuda")
    y8t = torch.empty(N, T, dtype=torch.float8_e4m3fn, device="cuda")
    # bytes: x, d read; sum written; y8 written, re-read and written transposed
    arms["add_rmsnorm_cast_t"] = (lambda: h.add_rmsnorm_cast_fp8_t(xx, dd, ww, 1e-5, s, y8, y8t, am),
                                  T * N * (2 + 2 + 2 + 1 + 1 + 1))
    t = {k: [] for k in arms}
    for _ in range(3):
        for k, (fn, _) in arms.items():
            t[k].append(timeit(fn))
    for k, (_, nbytes) in arms.items():
        m = statistics.median(t[k])
        print(json.dumps({"shape": [T, F], "op": k, "us": round(m * 1e3, 1), "TBps": round(nbytes / m / 1e9, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
