"""LM-head forward (logits = h W^T) and input gradient (dh = dlogits W) on hipBLASLt (with the config's TunableOp
table, as bench.py loads it) against the hand ping-pong kernel (``gemm_pp``, both operands K-major), per config.

    python benchmarks/head_routes.py [--configs llama-1.1b:65536:32000:2048,gpt2-small:131072:50432:768]

Prints one JSON line per config: milliseconds (median of 5 rounds) and PF/s of each route, and the max relative
difference between the routes' outputs.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402

TUNING = {"llama-1.1b:65536": "llama-1.1b_b16_s4096.csv", "gpt2-small:131072": "gpt2-small_b128_s1024.csv"}


def timed(fn, reps=5):
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
    ap.add_argument("--configs", default="llama-1.1b:65536:32000:2048,gpt2-small:131072:50432:768")
    a = ap.parse_args()
    h = ops()
    import torch.cuda.tunable as tunable

    for cfg in a.configs.split(","):
        model, T, V, d = cfg.split(":")
        T, V, d = int(T), int(V), int(d)
        tab = TUNING.get(f"{model}:{T}")
        if tab:
            tunable.enable(True)
            tunable.tuning_enable(False)
            tunable.record_untuned_enable(False)
            tunable.read_file(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                           "bpe_transformer", "ops", "tuning", tab))
        torch.manual_seed(0)
        x = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(V, d, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = h.transpose_bf16(w)
        dl = torch.randn(T, V, device="cuda", dtype=torch.bfloat16) * 1e-3
        logits = torch.empty(T, V, device="cuda", dtype=torch.bfloat16)
        dh = torch.empty(T, d, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * V * d
        res = {"model": model, "tokens": T, "vocab": V, "d": d, "tuning": tab}
        arms = {
            "fwd_blas": lambda: torch.matmul(x, w.t(), out=logits),
            "fwd_pp": lambda: h.gemm_pp(x, True, w, True, logits, 0.0, 1),
            "dx_blas_tn": lambda: torch.matmul(dl, wt.t(), out=dh),
            "dx_pp": lambda: h.gemm_pp(dl, True, wt, True, dh, 0.0, 1),
        }
        outs = {}
        for k, fn in arms.items():
            fn()
            torch.cuda.synchronize()
            outs[k] = (logits if k.startswith("fwd") else dh).float().clone()
        for pre in ("fwd", "dx"):
            ks = [k for k in outs if k.startswith(pre)]
            r = outs[ks[0]]
            res[f"{pre}_maxrel"] = float((outs[ks[1]] - r).abs().max() / r.abs().max().clamp_min(1e-30))
        del outs
        for k, fn in arms.items():
            ms = timed(fn)
            res[f"{k}_ms"] = round(ms, 3)
            res[f"{k}_pfs"] = round(fl / ms / 1e12, 3)
        print(json.dumps(res), flush=True)
        tunable.enable(False)


if __name__ == "__main__":
    main()
