"""The fp8 W13 projection with the SwiGLU gate and its two-layout e4m3 cast fused into the hand kernel's epilogue
(``gemm_fp8_swiglu``, gemm_pp.hip EPI_SWIGLU_FWD8) against the unfused pair the fp8 path ran before: the W13 GEMM
(hipBLASLt ``_scaled_mm``, or the hand kernel) then ``swiglu_cast_fp8_t`` over gu; and the backward: the W2 input
gradient with the SwiGLU backward + e5m2 two-layout cast fused (``gemm_fp8_swiglu_bwd``, EPI_SWIGLU_BWD8) against
``_scaled_mm`` then ``swiglu_cast_fp8_t(gu, da)``.  Llama-1.1B widths.

    python benchmarks/fp8_swiglu_gemm.py [--tokens 65536]

One JSON line: median ms of each arm (interleaved rounds).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--d", type=int, default=2048)
    ap.add_argument("--ff", type=int, default=5632)
    a = ap.parse_args()
    h = ops()
    M, K, F = a.tokens, a.d, a.ff
    torch.manual_seed(0)
    x8 = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
    w8 = (4 * torch.randn(2 * F, K, device="cuda")).to(torch.float8_e4m3fn)
    sx = torch.tensor([0.25], device="cuda")
    sw = torch.tensor([1.0 / (K**0.5)], device="cuda")
    sc = torch.tensor([4.0], device="cuda")
    amax = torch.zeros(1, dtype=torch.int32, device="cuda")
    a8 = torch.empty(M, F, dtype=torch.float8_e4m3fn, device="cuda")
    a8t = torch.empty(F, M, dtype=torch.float8_e4m3fn, device="cuda")

    def lib_then_cast():
        gu = torch._scaled_mm(x8, w8.t(), scale_a=sx[0], scale_b=sw[0], out_dtype=torch.bfloat16)
        h.swiglu_cast_fp8_t(gu, None, sc, a8, a8t, amax)

    def hip_then_cast():
        gu = h.gemm_fp8(x8, w8, sx, sw)
        h.swiglu_cast_fp8_t(gu, None, sc, a8, a8t, amax)

    arms = {"lib_gemm_then_cast": lib_then_cast, "hip_gemm_then_cast": hip_then_cast,
            "fused": lambda: h.gemm_fp8_swiglu(x8, w8, sx, sw, sc, a8, a8t, amax),
            "lib_gemm_only": lambda: torch._scaled_mm(x8, w8.t(), scale_a=sx[0], scale_b=sw[0],
                                                      out_dtype=torch.bfloat16)}
    # backward: da = g8 @ W2 (e5m2 x e4m3) then the SwiGLU backward + e5m2 two-layout cast, vs fused
    g8 = torch.randn(M, K, device="cuda").to(torch.float8_e5m2)
    w2t8 = (4 * torch.randn(F, K, device="cuda")).to(torch.float8_e4m3fn)
    gu = torch.randn(M, 2 * F, device="cuda").to(torch.bfloat16)
    d8 = torch.empty(M, 2 * F, dtype=torch.float8_e5m2, device="cuda")
    d8t = torch.empty(2 * F, M, dtype=torch.float8_e5m2, device="cuda")
    dsc = torch.tensor([64.0], device="cuda")

    def bwd_lib_then_cast():
        da = torch._scaled_mm(g8, w2t8.t(), scale_a=sx[0], scale_b=sw[0], out_dtype=torch.bfloat16)
        h.swiglu_cast_fp8_t(gu, da, dsc, d8, d8t, amax)

    arms["bwd_lib_gemm_then_cast"] = bwd_lib_then_cast
    arms["bwd_fused"] = lambda: h.gemm_fp8_swiglu_bwd(g8, w2t8, sx, sw, gu, dsc, d8, d8t, amax)
    arms["bwd_lib_gemm_only"] = lambda: torch._scaled_mm(g8, w2t8.t(), scale_a=sx[0], scale_b=sw[0],
                                                         out_dtype=torch.bfloat16)
    for f in arms.values():
        f()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {k: [] for k in arms}
    for _ in range(5):
        for k, f in arms.items():
            f()
            ev[0].record()
            for _ in range(3):
                f()
            ev[1].record()
            torch.cuda.synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]) / 3)
    print(json.dumps({"M": M, "K": K, "F": F, **{k + "_ms": round(statistics.median(v), 4) for k, v in times.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
