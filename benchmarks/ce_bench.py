"""Fused softmax-CE (forward loss + in-place gradient) microbenchmark at the LM-head shape.

Reports the kernel time and the effective HBM rate (one read + one write of the logits)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--ld", type=int, default=50432)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    buf = torch.randn(a.rows, a.ld, device="cuda", dtype=torch.bfloat16)
    t = torch.randint(0, a.vocab, (a.rows,), device="cuda")
    ops().ce_fwd_bwd(buf[:, : a.vocab], t, -100, True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        ops().ce_fwd_bwd(buf[:, : a.vocab], t, -100, True)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / a.iters
    gb = 2 * a.rows * a.vocab * 2 / 1e9
    print(json.dumps({"rows": a.rows, "vocab": a.vocab, "ms": round(ms, 3), "TB_s": round(gb / ms, 2)}))


if __name__ == "__main__":
    main()
