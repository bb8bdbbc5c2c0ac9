"""The plain (no-epilogue) forward and input-gradient GEMMs of a block: hipBLASLt (the bench's TunableOp table, the
layouts fused_block.py uses) against the persistent ping-pong kernel (gemm_pp.hip, auto tile order).

    python benchmarks/plain_gemm_routes.py --model gpt2-small|llama-1.1b

One JSON line per GEMM: median ms of interleaved repetitions for ``lib`` and ``pp`` (K-major B) / ``pp_mn``
(the weight as an MN-major B, no transposed copy), and the max relative difference of pp to lib.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402

SHAPES = {  # name: (tokens, d, d_ff, qkv width, vocab, TunableOp table)
    "gpt2-small": (131072, 768, 2048, 2304, 50432, "gpt2-small_b128_s1024.csv"),
    "llama-1.1b": (65536, 2048, 5632, 2560, 32000, "llama-1.1b_b32_s2048.csv"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small", choices=list(SHAPES))
    ap.add_argument("--head", action="store_true", help="also the LM-head GEMMs (13 GB of logits at GPT-2)")
    a = ap.parse_args()
    T, d, F, NQ, V, table = SHAPES[a.model]
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    tunable.read_file(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bpe_transformer",
                                   "ops", "tuning", table))
    h = ops()
    # (name, x rows, in width, out width, kind): fwd y = x W^T (W [out][in]); dx: dX = g W (W [out][in], g [T][out])
    gemms = [("o_fwd", d, d, "fwd"), ("w2_fwd", F, d, "fwd"), ("qkv_dx", NQ, d, "dx"), ("w13_dx", 2 * F, d, "dx"),
             ("o_dx", d, d, "dx")]
    if a.head:
        gemms += [("head_fwd", d, V, "fwd"), ("head_dx", V, d, "dx")]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, n_in, n_out, kind in gemms:
        torch.manual_seed(0)
        if kind == "fwd":  # x [T][n_in], W [n_out][n_in] -> y [T][n_out]
            x = torch.randn(T, n_in, device="cuda", dtype=torch.bfloat16)
            w = (0.05 * torch.randn(n_out, n_in, device="cuda")).to(torch.bfloat16)
            c = torch.empty(T, n_out, device="cuda", dtype=torch.bfloat16)
            arms = {"lib": lambda: torch.matmul(x, w.t(), out=c),
                    "pp": lambda: h.gemm_pp(x, True, w, True, c, 0.0, 1)}
        else:  # g [T][n_in] (n_in = the projection's output width), W [n_in][n_out] -> dX [T][n_out]
            x = torch.randn(T, n_in, device="cuda", dtype=torch.bfloat16)
            w = (0.05 * torch.randn(n_in, n_out, device="cuda")).to(torch.bfloat16)
            wt = h.transpose_bf16(w)
            c = torch.empty(T, n_out, device="cuda", dtype=torch.bfloat16)
            arms = {"lib": lambda: torch.matmul(x, w, out=c), "lib_tn": lambda: torch.matmul(x, wt.t(), out=c),
                    "pp": lambda: h.gemm_pp(x, True, wt, True, c, 0.0, 1),
                    "pp_mn": lambda: h.gemm_pp(x, True, w, False, c, 0.0, 1)}
        outs = {}
        for k, f in arms.items():
            f()
            torch.cuda.synchronize()
            outs[k] = c.float().clone()
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
        ref = outs["lib"]
        res = {"model": a.model, "gemm": name, "T": T, "in": n_in, "out": n_out}
        for k in arms:
            res[k + "_ms"] = round(statistics.median(times[k]), 4)
            res[k + "_maxrel"] = round(float((outs[k] - ref).abs().max() / ref.abs().max()), 5)
        print(json.dumps(res), flush=True)
        del x, w, c, outs


if __name__ == "__main__":
    main()
