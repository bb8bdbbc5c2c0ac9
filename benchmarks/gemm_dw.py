"""Weight-gradient GEMM microbenchmark (dW += dY^T X) at the GPT-2-small and Llama-1.1B shapes:
hipBLASLt vs the 256-tile kernel (routing of ops.gemm), TFLOP/s.  Set BPE_G256_VARIANT to A/B kernel
variants (one per process)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops as hip  # noqa: E402
from bpe_transformer.ops.gemm import choose_splits_256  # noqa: E402

SHAPES = {"gpt2": (65536, [(2304, 768), (768, 768), (4096, 768), (768, 2048)]),
          "llama": (16384, [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632)])}


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


def sweep():
    """ms per split count for each GPT-2 dW shape (incl. the padded LM head), 256-tile kernel."""
    T = 65536
    for n, k in SHAPES["gpt2"][1] + [(50432, 768)]:
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        res = {}
        for sp in sorted({1, 2, 3, 4, 5, 6, 8, 9, 10, 12, 14, 16, 20, 24, 28, 32, choose_splits_256(n, k, T)}):
            if (n // 256) * (k // 256) * sp > 8 * 256:
                continue
            res[sp] = round(statistics.median(bench(lambda: hip().gemm(dy, False, x, False, g, 1.0, sp, 256))
                                              for _ in range(3)), 4)
        best = min(res, key=res.get)
        fl = 2.0 * n * k * T
        print(json.dumps({"shape": [n, k], "model_splits": choose_splits_256(n, k, T), "best_splits": best,
                          "best_tf": round(fl / res[best] / 1e9), "ms": res}), flush=True)
        del dy, x, g


def layouts():
    """GPT-2 B 128 dW shapes (T = 131072): the 256-tile kernel at its model split count, the ping-pong kernel on
    the same token-major operands over a split sweep, and the ping-pong kernel on K-major copies of both operands
    (dY^T, X^T: what the loop reaches when no operand is read transposed), TFLOP/s."""
    from bpe_transformer.ops.gemm import choose_splits_pp
    T = 131072
    for n, k in SHAPES["gpt2"][1]:
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        dyt, xt = dy.t().contiguous(), x.t().contiguous()
        g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * n * k * T
        tf = lambda fn: round(fl / statistics.median(bench(fn) for _ in range(3)) / 1e9)  # noqa: E731
        row = {"shape": [n, k, T], "hip256": tf(lambda: hip().gemm(dy, False, x, False, g, 1.0,
                                                                    choose_splits_256(n, k, T), 256)),
               "pp_model_splits": choose_splits_pp(n, k, T)}
        for sp in sorted({choose_splits_pp(n, k, T), 4, 8, 12, 16, 24, 32}):
            if (n // 256) * (k // 256) * sp > 4 * 256:
                continue
            row[f"pp_mn_s{sp}"] = tf(lambda: hip().gemm_pp(dy, False, x, False, g, 1.0, sp))
            row[f"pp_kmajor_s{sp}"] = tf(lambda: hip().gemm_pp(dyt, True, xt, True, g, 1.0, sp))
        print(json.dumps(row), flush=True)
        del dy, x, dyt, xt, g


def main():
    if "--sweep" in sys.argv:
        return sweep()
    if "--layouts" in sys.argv:
        return layouts()
    out = {"variant": os.environ.get("BPE_G256_VARIANT", "0")}
    for model, (T, shapes) in SHAPES.items():
        tot_b = tot_o = 0.0
        for n, k in shapes:
            dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
            x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
            g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
            sp = choose_splits_256(n, k, T)
            tb, to = [], []
            for _ in range(3):
                tb.append(bench(lambda: g.addmm_(dy.t(), x)))
                to.append(bench(lambda: hip().gemm(dy, False, x, False, g, 1.0, sp, 256)))
            mb, mo = statistics.median(tb), statistics.median(to)
            fl = 2.0 * n * k * T
            out[f"{model}_{n}x{k}"] = {"blas_tf": round(fl / mb / 1e9), "ours_tf": round(fl / mo / 1e9), "splits": sp}
            tot_b += mb
            tot_o += mo
        out[f"{model}_layer_ms"] = {"blas": round(tot_b, 4), "ours": round(tot_o, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
