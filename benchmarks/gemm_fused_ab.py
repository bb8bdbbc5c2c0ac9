"""Time the fused ping-pong GEMMs of one GPT-2-small (or Llama) layer -- SwiGLU forward, SwiGLU backward, QKV with
RoPE -- and the fp8 hand kernel on the same shapes, for A/B runs of library variants (``BPE_HIP_VARIANT``).

    python benchmarks/gemm_fused_ab.py [--tokens 131072] [--d 768] [--ff 2048] [--reps 20]

Prints one JSON line: microseconds per call of each GEMM (median of 5 rounds of ``reps`` calls).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops import reference as R  # noqa: E402
from bpe_transformer.ops._ext import ops  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    out = []
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(5):
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        out.append(ev[0].elapsed_time(ev[1]) * 1000.0 / reps)
    return sorted(out)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--ff", type=int, default=2048)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    h = ops()
    T, d, F, S = a.tokens, a.d, a.ff, a.seq
    torch.manual_seed(0)
    x = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)
    w13 = torch.randn(2 * F, d, device="cuda", dtype=torch.bfloat16) * 0.05
    w2 = torch.randn(d, F, device="cuda", dtype=torch.bfloat16) * 0.05
    wqkv = torch.randn(3 * d, d, device="cuda", dtype=torch.bfloat16) * 0.05
    dy = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)
    D = 64
    cos, sin = R.rope_tables(D, S, 10000.0, device="cuda")
    gu, _ = h.gemm_swiglu_fwd(x, w13)
    res = {"variant": os.environ.get("BPE_HIP_VARIANT"), "tokens": T, "d": d, "ff": F}
    res["swiglu_fwd_us"] = round(timed(lambda: h.gemm_swiglu_fwd(x, w13), a.reps), 1)
    res["swiglu_bwd_us"] = round(timed(lambda: h.gemm_swiglu_bwd(dy, w2, gu), a.reps), 1)
    res["qkv_rope_us"] = round(timed(lambda: h.gemm_qkv_rope(x, wqkv, cos, sin, S, D, 2 * d), a.reps), 1)
    c = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    res["w13_plain_us"] = round(timed(lambda: h.gemm_pp(x, True, w13, True, c, 0.0, 1), a.reps), 1)
    # fp8 (e4m3 x e4m3) on the W13 shape
    x8 = (x * 4).to(torch.float8_e4m3fn)
    w8 = (w13 * 64).to(torch.float8_e4m3fn)
    one = torch.ones(1, device="cuda")
    res["fp8_w13_us"] = round(timed(lambda: h.gemm_fp8(x8, w8, one, one), a.reps), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
