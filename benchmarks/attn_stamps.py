"""Per-workgroup phase times of the split attention backward from in-kernel s_memtime stamps.

Needs the stamps variant build (``python -m bpe_transformer.ops.build --variant stamps -D BPE_FA_STAMPS``) and runs
with ``BPE_HIP_VARIANT=stamps``.  For each kernel (dQ, dK/dV) and each tile count it prints the mean workgroup
duration, its prologue (entry -> first barrier) and the time per full tile and the last (diagonal) tile, in shader cycles.
usage: BPE_HIP_VARIANT=stamps python benchmarks/attn_stamps.py [--batch B] [--seq S] [--heads H] [--kv-heads Hkv]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops import reference as R  # noqa: E402
from bpe_transformer.ops._ext import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--kv-heads", type=int, default=None)
    ap.add_argument("--dq-form", type=int, default=0, help="ops.fa_dq_config: 0 = 32 queries per wave, 1 = 16 (8 waves), 2 = 16 (4 waves), 3 = auto")
    a = ap.parse_args()
    h = ops()
    h.fa_dq_config(a.dq_form)
    B, S, H, D = a.batch, a.seq, a.heads, 64
    Hkv = a.kv_heads or H
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    cos, sin = R.rope_tables(D, S, 10000.0, device="cuda")
    h.rope_qk_(qkv, cos, sin, B, S, H, Hkv, D)
    q, k, v = qkv[:, : H * D], qkv[:, H * D : (H + Hkv) * D], qkv[:, (H + Hkv) * D :]
    o, lse = h.fa_fwd(q, k, v, cos, sin, B, S, H, Hkv, D, True, True, D ** -0.5, True)
    do = torch.randn_like(o)
    for _ in range(3):
        h.fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, True, True, D ** -0.5, True)
    torch.cuda.synchronize()
    st = h.fa_stamps(65536).double()
    if st.numel() == 0:
        sys.exit("not a BPE_FA_STAMPS build: set BPE_HIP_VARIANT=stamps (ops.build --variant stamps -D BPE_FA_STAMPS)")
    nblk = (S + 127) // 128
    qb = 64 if a.dq_form == 2 else 128  # queries per dQ workgroup
    for name, base, n in (("dQ", 0, min(32768, (S + qb - 1) // qb * B * H)), ("dK/dV", 32768, nblk * B * Hkv)):
        r = st[base : base + n]
        # slot 2 = start of the last (diagonal) tile; the epilogue is not stamped (entry .. slot 3)
        dur, pro, nt = r[:, 3] - r[:, 0], r[:, 1] - r[:, 0], r[:, 5]
        diag, body = r[:, 3] - r[:, 2], r[:, 2] - r[:, 1]
        print(f"{name} B={B} S={S} H={H} Hkv={Hkv} dq_form={a.dq_form}: {n} workgroups, mean {dur.mean():.0f} cycles: "
              f"prologue {pro.mean():.0f} ({pro.sum() / dur.sum() * 100:.1f} %), full tiles {body.mean():.0f} "
              f"({body.sum() / dur.sum() * 100:.1f} %), last (diagonal) tile {diag.mean():.0f} "
              f"({diag.sum() / dur.sum() * 100:.1f} %)")
        if name == "dQ" and a.dq_form in (1, 2):  # slots 6 (loads issued) and 4 (the wave's row loads arrived)
            iss, rows = r[:, 6] - r[:, 0], r[:, 4] - r[:, 0]
            print(f"  prologue split (last wave): loads issued at {iss.mean():.0f}, its rows arrived at {rows.mean():.0f}, "
                  f"barrier (tile-0 DMA, all waves) passed at {pro.mean():.0f} cycles after entry")
        for t in sorted(set(nt.tolist())):
            m = nt == t
            full = (body[m] / (t - 1)).mean() if t > 1 else float("nan")
            print(f"  tiles {int(t):3d}: n {int(m.sum()):5d}  workgroup {dur[m].mean():8.0f}  prologue {pro[m].mean():6.0f}"
                  f"  full tile {full:6.0f}  last tile {diag[m].mean():6.0f}")


if __name__ == "__main__":
    main()
