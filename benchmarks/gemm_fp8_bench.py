"""Hand-written fp8 GEMM (``csrc/gemm_pp.hip`` F8 variants: ping-pong kernel on v_mfma_scale_f32_16x16x128_f8f6f4)
against hipBLASLt's ``torch._scaled_mm`` and bf16 ``torch.matmul`` on the Llama-1.1B projection shapes (16384
tokens: forward Y = X W^T, and the input gradient dX = dY W in the K-major form the fp8 path uses).  Random
normal data; interleaved rounds in one process (guide §5.4 rule 24), median ms and TF/s per arm."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402

SHAPES = {  # name: (M, N, K)
    "qkv_fwd": (16384, 2560, 2048), "o_fwd": (16384, 2048, 2048), "w13_fwd": (16384, 11264, 2048),
    "w2_fwd": (16384, 2048, 5632), "qkv_dx": (16384, 2048, 2560), "w13_dx": (16384, 2048, 11264),
    "w2_dx": (16384, 5632, 2048), "gpt2_qkv_fwd": (131072, 2304, 768),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=16384,
                    help="M of the Llama shapes (16384 = s4096 B4; 65536 = s4096 B16, the bench default)")
    ap.add_argument("--orders", type=int, nargs="*", default=[], help="extra hand-kernel arms at these tile orders")
    a = ap.parse_args()
    h = ops()
    for name, (M, N, K) in SHAPES.items():
        if not name.startswith("gpt2"):
            M = a.tokens
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        fa = torch.float8_e5m2 if name.endswith("_dx") else torch.float8_e4m3fn  # dgrad: e5m2 gradient
        x8, w8 = x.to(fa), w.to(torch.float8_e4m3fn)
        one = torch.ones(1, device="cuda")
        arms = {
            "hip_fp8": lambda: (h.gpp_order_config(0), h.gemm_fp8(x8, w8, one, one))[1],
            "lib_fp8": lambda: torch._scaled_mm(x8, w8.t(), scale_a=one[0], scale_b=one[0], out_dtype=torch.bfloat16),
            "bf16": lambda: x @ w.t(),
        }
        for gm in a.orders:  # the hand kernel under explicit column-major tile orders (gemm_pp.hip tile_rc)
            arms[f"hip_fp8_gm{gm}"] = (lambda gm=gm: (h.gpp_order_config(gm), h.gemm_fp8(x8, w8, one, one))[1])
        ref = x8.float() @ w8.float().t()
        err = float(((h.gemm_fp8(x8, w8, one, one).float() - ref).norm() / ref.norm()).item())
        times = {k: [] for k in arms}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(a.rounds):
            for k, f in arms.items():
                f()
                ev[0].record()
                for _ in range(a.iters):
                    f()
                ev[1].record()
                torch.cuda.synchronize()
                times[k].append(ev[0].elapsed_time(ev[1]) / a.iters)
        row = {"shape": name, "MNK": [M, N, K], "hip_fp8_rel_err": round(err, 6)}
        for k, t in times.items():
            med = sorted(t)[len(t) // 2]
            row[f"{k}_ms"] = round(med, 4)
            row[f"{k}_tflops"] = round(2 * M * N * K / med / 1e9, 1)
        print(json.dumps(row), flush=True)


def wgrad(a) -> None:
    """Weight-gradient GEMMs dW = dY^T X of the Llama projections: fp8 (e5m2 dY^T x e4m3 X^T, both [., tokens],
    hipBLASLt) against the bf16 route the model takes (ops.gemm.accumulate_weight_grad)."""
    from bpe_transformer.ops.gemm import accumulate_weight_grad

    for name, (n, k) in {"qkv_dw": (2560, 2048), "o_dw": (2048, 2048), "w13_dw": (11264, 2048),
                         "w2_dw": (2048, 5632)}.items():
        T = a.tokens
        g = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        gt8 = g.t().contiguous().to(torch.float8_e5m2)
        xt8 = x.t().contiguous().to(torch.float8_e4m3fn)
        one = torch.ones(1, device="cuda")
        acc = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        from bpe_transformer.ops.gemm import choose_splits_pp

        sp = choose_splits_pp(n, k, T // 2)
        arms = {
            "lib_fp8": lambda: torch._scaled_mm(gt8, xt8.t(), scale_a=one[0], scale_b=one[0],
                                                out_dtype=torch.bfloat16),
            "lib_fp8_acc": lambda: acc.add_(torch._scaled_mm(gt8, xt8.t(), scale_a=one[0], scale_b=one[0],
                                                             out_dtype=torch.bfloat16)),
            "hip_fp8_splitk_acc": lambda: ops().gemm_fp8_acc(gt8, xt8, one, one, acc, 1.0, sp),
            "bf16_route": lambda: accumulate_weight_grad(acc, g, x),
        }
        ref = gt8.float() @ xt8.float().t()
        acc.zero_()
        ops().gemm_fp8_acc(gt8, xt8, one, one, acc, 1.0, sp)
        err = float(((acc.float() - ref).norm() / ref.norm()).item())
        times = {kk: [] for kk in arms}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(a.rounds):
            for kk, f in arms.items():
                f()
                ev[0].record()
                for _ in range(a.iters):
                    f()
                ev[1].record()
                torch.cuda.synchronize()
                times[kk].append(ev[0].elapsed_time(ev[1]) / a.iters)
        row = {"shape": name, "NKT": [n, k, T], "splits": sp, "hip_rel_err": round(err, 5)}
        for kk, t in times.items():
            med = sorted(t)[len(t) // 2]
            row[f"{kk}_ms"] = round(med, 4)
            row[f"{kk}_tflops"] = round(2 * n * k * T / med / 1e9, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    if "--wgrad" in sys.argv:
        sys.argv.remove("--wgrad")
        ap = argparse.ArgumentParser()
        ap.add_argument("--iters", type=int, default=10)
        ap.add_argument("--rounds", type=int, default=3)
        ap.add_argument("--tokens", type=int, default=65536)
        wgrad(ap.parse_args())
    else:
        main()
