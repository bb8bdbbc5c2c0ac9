"""Weight-gradient GEMM dW += dY^T X through hipBLASLt as a K-split batched GEMM, against the hand-written route.

hipBLASLt alone does not split the token reduction (280-850 TF/s on these shapes, docs/performance.md).  Here the
tokens are cut into ``s`` chunks and the chunks run as ONE strided-batched GEMM with an fp32 output
(``torch.bmm(..., out_dtype=torch.float32)``: s partial [N, K] products, no bf16 rounding of a partial), then the
partials are summed in batch order into g -- the same split-K scheme as the hand-written kernel, with the
library's GEMM core.

    python benchmarks/dw_bmm.py [--tokens 131072]

One JSON line per shape: ms of the hand-written route (``pp`` at the cost model's split) and of the batched form
at each split count (the reduce included), and the max relative difference to the hand route's result.
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
    shapes = [("qkv", 2304, 768), ("o", 768, 768), ("w13", 4096, 768), ("w2", 768, 2048), ("head", 50432, 768)]
    for name, n, k in shapes:
        torch.manual_seed(0)
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16) * 0.01
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        sp = choose_splits_pp(n, k, T)
        res = {"shape": name, "N": n, "K": k, "T": T, "pp_splits": sp}
        fn = lambda: h.gemm_pp(dy, False, x, False, g, 1.0, sp)  # noqa: E731
        ms = timed(fn)
        res["pp_ms"] = round(ms, 4)
        res["pp_tf"] = round(2 * n * k * T / ms / 1e9, 1)
        gref = torch.zeros_like(g)
        h.gemm_pp(dy, False, x, False, gref, 1.0, sp)
        for s in (2, 4, 8, 16):
            tc = T // s
            dyb = dy.view(s, tc, n).transpose(1, 2)  # [s, N, tc], no copy
            xb = x.view(s, tc, k)

            def bfn():
                p = torch.bmm(dyb, xb, out_dtype=torch.float32)
                g.add_(p.sum(0).to(torch.bfloat16))

            try:
                ms = timed(bfn)
            except (RuntimeError, TypeError) as e:
                res[f"bmm{s}_ms"] = str(e).splitlines()[0][:100]
                continue
            gb = torch.zeros_like(g)
            gb.add_(torch.bmm(dyb, xb, out_dtype=torch.float32).sum(0).to(torch.bfloat16))
            res[f"bmm{s}_ms"] = round(ms, 4)
            res[f"bmm{s}_tf"] = round(2 * n * k * T / ms / 1e9, 1)
            res[f"bmm{s}_maxrel"] = float((gb.float() - gref.float()).abs().max() / gref.float().abs().max())
            # the batched GEMM alone (no reduce)
            res[f"bmm{s}_gemm_ms"] = round(timed(lambda: torch.bmm(dyb, xb, out_dtype=torch.float32)), 4)
        print(json.dumps(res), flush=True)
        del dy, x, g, gref


if __name__ == "__main__":
    main()
