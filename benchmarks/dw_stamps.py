"""Where the weight-gradient GEMMs lose time: per-workgroup timelines of the ping-pong kernel's split-K form.

Needs the stamps variant build (``python -m bpe_transformer.ops.build --variant stamps -D BPE_GPP_STAMPS``) and
runs with ``BPE_HIP_VARIANT=stamps``.  For every GPT-2 B 128 dW shape (dW += dY^T X, both operands token-major, the
``pp`` route) and a few split counts it launches the one-tile kernel once more after warm-up, reads the per-workgroup
``s_memtime`` stamps (entry, K-tile 0 retired, main loop done, slab stores issued, XCC id, CU id) and prints, per
shape and split count, in shader cycles:

* ``kt``: main-loop cycles per 64-deep K-tile (mean over workgroups), against ``mfma`` = 2 048 cycles of MFMA issue;
* ``pro`` / ``epi``: prologue and slab-store cycles per workgroup;
* ``busy``: the summed workgroup time of an XCD over (its span x its CUs): what wave quantisation, the tail and the
  gaps between a CU's workgroups cost;
* ``span``: the mean per-XCD kernel span, and ``ms``: the op's wall time (CUDA events, slab reduce included).

    BPE_HIP_VARIANT=stamps python benchmarks/dw_stamps.py [--tokens 131072]
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


def analyse(st: torch.Tensor, n: int, nk_mean: float) -> dict:
    r = st[:n].double()
    pro, loop, epi = r[:, 1] - r[:, 0], r[:, 2] - r[:, 1], r[:, 4] - r[:, 2]
    xcc = r[:, 7].long()
    cu = (r[:, 5].long() >> 8) & 0x7F
    busy, spans, tails = [], [], []
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        rx = r[m]
        span = rx[:, 4].max() - rx[:, 0].min()
        ncu = len(set(cu[m].tolist()))
        busy.append(((rx[:, 4] - rx[:, 0]).sum() / (span * ncu)).item())
        spans.append(span.item())
        # tail: from the first CU of this XCD going idle for good to the XCD's last store
        last_per_cu = [rx[cu[m] == c][:, 4].max().item() for c in set(cu[m].tolist())]
        tails.append(max(last_per_cu) - min(last_per_cu))
    return {"wgs": n, "kt": round(loop.mean().item() / nk_mean), "kt_min": round((loop / nk_mean).min().item()),
            "kt_max": round((loop / nk_mean).max().item()), "pro": round(pro.mean().item()),
            "epi": round(epi.mean().item()), "busy": round(statistics.mean(busy), 3),
            "span": round(statistics.mean(spans)), "tail": round(statistics.mean(tails))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--shapes", default="qkv,o,w13,w2,head")
    a = ap.parse_args()
    h = ops()
    T = a.tokens
    shapes = {"qkv": (2304, 768), "o": (768, 768), "w13": (4096, 768), "w2": (768, 2048), "head": (50432, 768)}
    for name in a.shapes.split(","):
        n, k = shapes[name]
        torch.manual_seed(0)
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16) * 0.01
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        tiles = (n // 256) * (k // 256)
        model = choose_splits_pp(n, k, T)
        cands = sorted({model, max(1, 256 // tiles), max(1, 512 // tiles), max(1, 768 // tiles)})
        for s in cands:
            if (T // 64) // s < 4 or tiles * s > 65536:
                continue
            fn = lambda: h.gemm_pp(dy, False, x, False, g, 1.0, s)  # noqa: E731
            ms = timed(fn)
            fn()
            torch.cuda.synchronize()
            st = h.gpp_stamps(65536)
            if st.numel() == 0:
                sys.exit("not a BPE_GPP_STAMPS build: set BPE_HIP_VARIANT=stamps "
                         "(ops.build --variant stamps -D BPE_GPP_STAMPS)")
            res = {"shape": name, "N": n, "K": k, "T": T, "tiles": tiles, "splits": s, "model": s == model,
                   "ms": round(ms, 4), "tflops": round(2 * n * k * T / ms / 1e9, 1)}
            res.update(analyse(st, tiles * s, (T // 64) / s))
            res["mhz_est"] = round(res["span"] / (ms * 1e3))
            print(json.dumps(res), flush=True)
        del dy, x, g


if __name__ == "__main__":
    main()
