"""Weight-gradient GEMM orientation on the ping-pong kernel: dW = dY^T X computed as itself with X transposed
(``ppt``: A = dY token-major = MN-major, B = X^T K-major -- the MN x K layout) or as its transpose dW^T = X^T dY
(A = X^T K-major, B = dY MN-major -- the K x MN layout, 1-6 % faster per K-tile in round 4's layout sweep,
profiles/bench/gemm_pp_layouts_r4.log), whose [K][N] result must then be added transposed into the [N][K]
gradient (one fp32 pass here: tmp written by the split-K reduce, then ``g += tmp^T`` rounded once).

    python benchmarks/dw_orient.py [--tokens 131072]

One JSON line per shape: ms of each form (X^T transpose included in both; the transposed add included in the
second) and the max relative difference of the two results.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402
from bpe_transformer.ops.gemm import choose_splits_pp  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    out = []
    for _ in range(5):
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        out.append(ev[0].elapsed_time(ev[1]) / reps)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    a = ap.parse_args()
    h = ops()
    T = a.tokens
    for name, n, k in [("head", 50432, 768), ("w13", 4096, 768), ("qkv", 2304, 768)]:
        torch.manual_seed(0)
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16) * 0.01
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        s = choose_splits_pp(n, k, T)
        g1 = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        g2 = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        tmp = torch.empty(k, n, device="cuda", dtype=torch.float32)

        def ppt():
            h.gemm_pp(dy, False, h.transpose_bf16(x), True, g1, 1.0, s)

        def kxmn():
            h.gemm_pp(h.transpose_bf16(x), True, dy, False, tmp, 0.0, s)
            g2.copy_((g2.float() + tmp.t()).to(torch.bfloat16))

        res = {"shape": name, "N": n, "K": k, "T": T, "splits": s}
        res["ppt_ms"] = round(timed(ppt), 4)
        res["kxmn_ms"] = round(timed(kxmn), 4)
        res["kxmn_gemm_only_ms"] = round(timed(lambda: h.gemm_pp(h.transpose_bf16(x), True, dy, False, tmp, 0.0, s)), 4)
        g1.zero_()
        g2.zero_()
        ppt()
        kxmn()
        res["maxrel"] = float((g1.float() - g2.float()).abs().max() / g1.float().abs().max())
        print(json.dumps(res), flush=True)
        del dy, x, g1, g2, tmp


if __name__ == "__main__":
    main()
