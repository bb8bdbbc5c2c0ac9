"""Flash-attention microbenchmark (fwd, bwd) on random data at training shapes; TFLOP/s counts the
causal half of the score matrix (fwd 4*B*H*S^2*D/2, bwd 2.5x that)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer import ops  # noqa: E402
from bpe_transformer.ops import reference as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--kv-heads", type=int, default=None)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-rope", action="store_true", help="plain attention (isolates the fused-RoPE cost)")
    a = ap.parse_args()
    B, S, H, D = a.batch, a.seq, a.heads, a.dim
    Hkv = a.kv_heads or H
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    cos, sin = (None, None) if a.no_rope else R.rope_tables(D, S, 10000.0, device="cuda")
    do = torch.randn(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        o = ops.flash_attention_qkv(qkv, B, S, H, Hkv, D, cos, sin, True)
        o.backward(do)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf, tb = 0.0, 0.0
    for _ in range(a.iters):
        e[0].record()
        o = ops.flash_attention_qkv(qkv, B, S, H, Hkv, D, cos, sin, True)
        e[1].record()
        o.backward(do)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    tf /= a.iters
    tb /= a.iters
    fl = 4.0 * B * H * S * S * D / 2
    print(json.dumps({"shape": [B, S, H, Hkv, D], "rope": not a.no_rope, "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4),
                      "fwd_tflops": round(fl / tf / 1e9, 1), "bwd_tflops": round(2.5 * fl / tb / 1e9, 1)}))


if __name__ == "__main__":
    main()
