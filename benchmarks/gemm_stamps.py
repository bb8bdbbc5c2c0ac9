"""Per-workgroup phase times of the ping-pong GEMM (gemm_pp.hip) from in-kernel s_memtime stamps.

Needs the stamps variant build (``python -m bpe_transformer.ops.build --variant stamps -D BPE_GPP_STAMPS``) and
runs with ``BPE_HIP_VARIANT=stamps``.  For each GEMM of a GPT-2-small layer at B 128 (fused SwiGLU forward and
backward, plain K-major forward GEMMs) it prints, in shader cycles, for both kernel forms (one tile per workgroup; persistent, stamped per tile), the mean prologue
(entry -> K-tile 0 retired; persistent: tile start -> main loop),
main loop, epilogue staging and store-issue times of a workgroup, the gap between consecutive workgroups of one
CU, and how many CUs of an XCD are issuing epilogue stores at the same time (in lock step: ~all of them; spread
evenly: the store share of the time times the CU count).
usage: BPE_HIP_VARIANT=stamps python benchmarks/gemm_stamps.py [--tokens T]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def analyse(name: str, st: torch.Tensor, n: int) -> None:
    r = st[:n].double()
    pro, loop, stage, store = r[:, 1] - r[:, 0], r[:, 2] - r[:, 1], r[:, 3] - r[:, 2], r[:, 4] - r[:, 3]
    tot = r[:, 4] - r[:, 0]
    print(f"{name}: {n} workgroups, mean {tot.mean():.0f} cycles = prologue {pro.mean():.0f} "
          f"({pro.sum() / tot.sum() * 100:.1f} %) + loop {loop.mean():.0f} ({loop.sum() / tot.sum() * 100:.1f} %) + "
          f"staging {stage.mean():.0f} ({stage.sum() / tot.sum() * 100:.1f} %) + stores {store.mean():.0f} "
          f"({store.sum() / tot.sum() * 100:.1f} %)")
    xcc = r[:, 7].long()
    cu = (r[:, 5].long() >> 8) & 0x7F
    gaps, conc, expect = [], [], []
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        rx = r[m]
        cux = cu[m]
        # consecutive workgroups (tiles) of one CU: entry of the next minus stores-issued of the previous
        for c in sorted(set(cux.tolist())):
            rc = rx[cux == c]
            rc = rc[rc[:, 0].argsort()]
            if rc.shape[0] > 1:
                gaps.append(rc[1:, 0] - rc[:-1, 4])
        # store-window overlap: for each workgroup, the number of workgroups of this XCD whose store window
        # contains the middle of its own
        mid = (rx[:, 3] + rx[:, 4]) / 2
        inside = (rx[None, :, 3] <= mid[:, None]) & (mid[:, None] <= rx[None, :, 4])
        conc.append(inside.sum(1).double())
        span = rx[:, 4].max() - rx[:, 0].min()
        ncu = len(set(cux.tolist()))
        expect.append(torch.tensor([((rx[:, 4] - rx[:, 3]).sum() / span).item(), float(ncu)]))
    g = torch.cat(gaps) if gaps else torch.zeros(1)
    c = torch.cat(conc)
    e = torch.stack(expect)
    print(f"  {len(set(xcc.tolist()))} XCDs x {e[:, 1].mean():.0f} CUs; gap between a CU's workgroups: mean "
          f"{g.mean():.0f}, median {g.median():.0f} cycles; CUs of an XCD storing at once: mean {c.mean():.1f} "
          f"(evenly spread would be {e[:, 0].mean():.1f})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--ff", type=int, default=2048)
    a = ap.parse_args()
    h = ops()
    T, d, F = a.tokens, a.d, a.ff
    torch.manual_seed(0)
    x = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)
    w13 = torch.randn(2 * F, d, device="cuda", dtype=torch.bfloat16) * 0.05
    w2 = torch.randn(d, F, device="cuda", dtype=torch.bfloat16) * 0.05
    wqkv = torch.randn(3 * d, d, device="cuda", dtype=torch.bfloat16) * 0.05
    dy = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)

    def run(fn, n, name):
        for mode in (0, 1):
            h.gpp_persist_config(mode)
            run1(fn, n, f"{name} [{'persistent' if mode else 'one tile'}]")
        h.gpp_persist_config(0)

    def run1(fn, n, name):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        st = h.gpp_stamps(65536)
        if st.numel() == 0:
            sys.exit("not a BPE_GPP_STAMPS build: set BPE_HIP_VARIANT=stamps "
                     "(ops.build --variant stamps -D BPE_GPP_STAMPS)")
        analyse(name, st, n)

    gu, _ = h.gemm_swiglu_fwd(x, w13)
    run(lambda: h.gemm_swiglu_fwd(x, w13), (T // 256) * (2 * F // 256), f"swiglu fwd T={T} d={d} F={F}")
    run(lambda: h.gemm_swiglu_bwd(dy, w2, gu), (T // 256) * (F // 256), f"swiglu bwd T={T} d={d} F={F}")
    c = torch.empty(T, 3 * d, device="cuda", dtype=torch.bfloat16)
    run(lambda: h.gemm_pp(x, True, wqkv, True, c, 0.0, 1), (T // 256) * (3 * d // 256), f"qkv fwd N={3 * d}")
    c2 = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    run(lambda: h.gemm_pp(x, True, w13, True, c2, 0.0, 1), (T // 256) * (2 * F // 256), f"w13 fwd plain N={2 * F}")


if __name__ == "__main__":
    main()
