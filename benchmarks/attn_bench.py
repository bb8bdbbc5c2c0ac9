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
    ap.add_argument("--no-causal", action="store_true", help="full (non-causal) attention")
    ap.add_argument("--bwd-ab", action="store_true",
                    help="interleaved same-process A/B of the backward forms (ops.fa_bwd_config / fa_dq_config): "
                         "fused (atomics), split, split with the 16-queries-per-wave dQ kernel")
    ap.add_argument("--fwd-ab", action="store_true",
                    help="interleaved same-process A/B of the D = 64 forward versions 2 (fa_fwd_kernel) and 8 "
                         "(flash_attn_fwd_v4.hip) (ops.fa_fwd_config)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dq-form", type=int, default=-1, help="ops.fa_dq_config form for the run (-1: the default)")
    ap.add_argument("--fwd-versions", type=int, nargs="+", default=[2, 8])
    ap.add_argument("--bwd-arms", nargs="+", default=None, help="subset of the --bwd-ab arms (names below)")
    ap.add_argument("--mode", choices=["block", "fused"], default="block",
                    help="block = the training path (rope_qk_ in place, then pre-rotated kernels; rope time reported "
                         "separately and included in fwd_ms); fused = RoPE inside the attention kernels")
    a = ap.parse_args()
    B, S, H, D = a.batch, a.seq, a.heads, a.dim
    Hkv = a.kv_heads or H
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    cos, sin = (None, None) if a.no_rope else R.rope_tables(D, S, 10000.0, device="cuda")
    do = torch.randn(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    from bpe_transformer.ops._ext import ops as _ops

    hip = _ops()
    if a.dq_form >= 0:
        hip.fa_dq_config(a.dq_form)
    scale = 1.0 / D ** 0.5
    rope = cos is not None
    causal = not a.no_causal
    pre = a.mode == "block" and rope
    x = qkv.detach().clone()
    q, k, v = x[:, : H * D], x[:, H * D : (H + Hkv) * D], x[:, (H + Hkv) * D :]
    c = cos if rope else torch.empty(0, 0, device="cuda")
    s_ = sin if rope else torch.empty(0, 0, device="cuda")

    def fwd():
        if pre:
            hip.rope_qk_(x, c, s_, B, S, H, Hkv, D)  # in place, as the fused block does (values drift: timing only)
        return hip.fa_fwd(q, k, v, c, s_, B, S, H, Hkv, D, causal, rope, scale, pre)

    def bwd(o, lse):
        return hip.fa_bwd(do, q, k, v, o, lse, c, s_, B, S, H, Hkv, D, causal, rope, scale, pre)

    for _ in range(3):
        o, lse = fwd()
        bwd(o, lse)
    torch.cuda.synchronize()
    fl = 4.0 * B * H * S * S * D / (1 if a.no_causal else 2)
    if a.fwd_ab:
        prev = hip.fa_fwd_config(0)
        times = {v: [] for v in a.fwd_versions}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(a.rounds):
            for ver in times:
                hip.fa_fwd_config(ver)
                hip.fa_fwd(q, k, v, c, s_, B, S, H, Hkv, D, causal, rope, scale, pre)
                ev[0].record()
                for _ in range(a.iters):
                    hip.fa_fwd(q, k, v, c, s_, B, S, H, Hkv, D, causal, rope, scale, pre)
                ev[1].record()
                torch.cuda.synchronize()
                times[ver].append(ev[0].elapsed_time(ev[1]) / a.iters)
        hip.fa_fwd_config(prev)
        for ver, t in times.items():
            t = sorted(t)
            print(json.dumps({"shape": [B, S, H, Hkv, D], "fwd_version": ver, "fwd_ms_median": round(t[len(t) // 2], 4),
                              "fwd_ms_min": round(t[0], 4), "fwd_tflops": round(fl / t[len(t) // 2] / 1e9, 1)}))
        if not a.bwd_ab:
            return
    if a.bwd_ab:
        # (backward form, dQ form): split with the 32- or 16-queries-per-wave dQ kernel (ops.fa_dq_config)
        # (backward form, dQ form)
        arms = {"fused": (1, 0), "split": (0, 0), "split_dq16": (0, 1), "split_dq16_nw4": (0, 2), "split_auto": (0, 3)}
        if a.bwd_arms:
            arms = {n: arms[n] for n in a.bwd_arms}
        prev = hip.fa_bwd_config(-1)
        prev_dq = hip.fa_dq_config(-1)
        times = {k: [] for k in arms}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(a.rounds):
            for name, (cfg, dqf) in arms.items():
                hip.fa_bwd_config(cfg)
                hip.fa_dq_config(dqf)
                bwd(o, lse)
                ev[0].record()
                for _ in range(a.iters):
                    bwd(o, lse)
                ev[1].record()
                torch.cuda.synchronize()
                times[name].append(ev[0].elapsed_time(ev[1]) / a.iters)
        hip.fa_bwd_config(prev)
        hip.fa_dq_config(prev_dq)
        for name, t in times.items():
            t = sorted(t)
            print(json.dumps({"shape": [B, S, H, Hkv, D], "arm": name, "bwd_ms_median": round(t[len(t) // 2], 4),
                              "bwd_ms_min": round(t[0], 4), "bwd_tflops": round(2.5 * fl / t[len(t) // 2] / 1e9, 1)}))
        return
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tf, tb, tr = 0.0, 0.0, 0.0
    for _ in range(a.iters):
        x.copy_(qkv.detach())
        e[0].record()
        if pre:
            hip.rope_qk_(x, c, s_, B, S, H, Hkv, D)
        e[3].record()
        o, lse = hip.fa_fwd(q, k, v, c, s_, B, S, H, Hkv, D, causal, rope, scale, pre)
        e[1].record()
        bwd(o, lse)
        e[2].record()
        torch.cuda.synchronize()
        tr += e[0].elapsed_time(e[3])
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    tf /= a.iters
    tb /= a.iters
    tr /= a.iters
    print(json.dumps({"shape": [B, S, H, Hkv, D], "rope": rope, "mode": a.mode, "rope_ms": round(tr, 4),
                      "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4),
                      "fwd_tflops": round(fl / tf / 1e9, 1), "bwd_tflops": round(2.5 * fl / tb / 1e9, 1)}))


if __name__ == "__main__":
    main()
