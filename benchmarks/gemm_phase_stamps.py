"""Where the ping-pong GEMM's K-tile goes: per-wave s_memtime stamps at every phase boundary and barrier arrival.

Needs the phase-stamps variant build (``python -m bpe_transformer.ops.build --variant pstamps -D
BPE_GPP_PHASE_STAMPS``) and runs with ``BPE_HIP_VARIANT=pstamps``.  The one-tile kernel (gemm_pp.hip, spread DMA
schedule) records, for K-tiles 2-5 of workgroups 0-1023, four events per phase and wave: 0 section start (before
the fragment reads), 1 after the wait (reads and this wave's DMA retired), 2 after the barrier (MFMA section
start), 3 after the last MFMA issued.  Group 1 (waves 4-7) runs one barrier behind group 0, so every barrier
closes an interval in which one group issued MFMAs and the other read fragments / issued DMA.

Printed per GEMM, in shader cycles (means over workgroups, waves, K-tiles):
  * per phase and group: load section (0 -> 1), barrier wait before the MFMAs (1 -> 2), MFMA issue (2 -> 3),
    barrier wait after them (3 -> next 0);
  * per barrier: which side arrives last -- the MFMA group's last issue or the loading group's wait -- and by how
    much (the loaders' lateness is time the matrix pipe has nothing queued from the partner);
  * the K-tile length against its 16 x 16 x 32 MFMA floor (4 x 2 x 16 MFMAs x 16 cycles = 2 048 per wave pair).
usage: BPE_HIP_VARIANT=pstamps python benchmarks/gemm_phase_stamps.py [--tokens T]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def analyse(name: str, st: torch.Tensor) -> dict:
    s = st.double()  # [wg, wave, kt, phase, event]
    s = s - s[:, :, :1, :1, :1].amin(dim=1, keepdim=True)  # per workgroup origin (any wave)
    n = s.shape[0]
    g0, g1 = s[:, :4], s[:, 4:]
    out = {"gemm": name, "workgroups": n}
    rows = []
    for gname, gs in (("group 0", g0), ("group 1", g1)):
        e = gs  # [wg, 4, kt, ph, ev]
        nxt0 = torch.cat([e[:, :, :, 1:, 0], torch.roll(e[:, :, :, :1, 0], -1, dims=2)], dim=3)  # next section start
        load = (e[..., 1] - e[..., 0])
        wb = (e[..., 2] - e[..., 1])
        mf = (e[..., 3] - e[..., 2])
        wa = (nxt0 - e[..., 3])[:, :, :-1]  # the last K-tile has no stamped successor
        for ph in range(4):
            rows.append((gname, ph, load[..., ph].mean().item(), wb[..., ph].mean().item(), mf[..., ph].mean().item(),
                         wa[..., ph].mean().item()))
    print(f"{name}: {n} workgroups, K-tiles 2-5")
    print("  group   phase  load   wait-before  MFMA-issue  wait-after   (cycles)")
    for r in rows:
        print(f"  {r[0]}  {r[1]}    {r[2]:6.0f}  {r[3]:6.0f}       {r[4]:6.0f}      {r[5]:6.0f}")
    # K-tile length: phase-0 section start of K-tile k+1 minus that of K-tile k, per wave
    kt_len = (s[:, :, 1:, 0, 0] - s[:, :, :-1, 0, 0]).mean().item()
    out["ktile_cycles"] = kt_len
    out["mfma_floor_share"] = 2048.0 / kt_len
    # barrier lateness.  Barrier "before the MFMAs of group 0, phase p": group 0 arrives at event 1 of (p), group 1
    # at event 3 of its phase p - 1 (it was issuing MFMAs); barrier "after group 0's MFMAs, phase p": group 0
    # arrives at event 3 of (p), group 1 at event 1 of (p) (its load section).
    late = []
    for p in range(4):
        a_g0 = g0[:, :, :, p, 1].amax(1)  # last loader of group 0 (before its MFMAs)
        if p > 0:
            a_g1 = g1[:, :, :, p - 1, 3].amax(1)
        else:
            a_g1 = torch.roll(g1[:, :, :, 3, 3].amax(1), 1, dims=1)
        d1 = (a_g0 - a_g1)[:, 1:] if p == 0 else (a_g0 - a_g1)
        late.append(("g0 loads / g1 MFMAs", p, d1.mean().item(), (d1 > 0).double().mean().item()))
        b_g0 = g0[:, :, :, p, 3].amax(1)  # group 0's last MFMA issue
        b_g1 = g1[:, :, :, p, 1].amax(1)  # group 1's last loader
        d2 = b_g1 - b_g0
        late.append(("g1 loads / g0 MFMAs", p, d2.mean().item(), (d2 > 0).double().mean().item()))
    print("  barrier (interval)         phase  loaders later than the MFMA group by (mean)  share of barriers")
    for r in late:
        print(f"  {r[0]:25s}  {r[1]}      {r[2]:8.0f}                                   {r[3] * 100:5.1f} %")
    print(f"  K-tile {kt_len:.0f} cycles; 16x16x32 MFMA floor 2048 ({out['mfma_floor_share'] * 100:.1f} % of it)")
    out["rows"] = rows
    out["late"] = late
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--ff", type=int, default=2048)
    a = ap.parse_args()
    h = ops()
    T, d, F = a.tokens, a.d, a.ff
    torch.manual_seed(0)
    h.gpp_persist_config(0)  # the stamps are taken by the one-tile kernel
    x = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)
    w13 = torch.randn(2 * F, d, device="cuda", dtype=torch.bfloat16) * 0.05
    xs = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    ws = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16) * 0.05

    def run(fn, name):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        st = h.gpp_phase_stamps(1024)
        if st.numel() == 0:
            sys.exit("not a BPE_GPP_PHASE_STAMPS build: set BPE_HIP_VARIANT=pstamps "
                     "(ops.build --variant pstamps -D BPE_GPP_PHASE_STAMPS)")
        analyse(name, st)

    c = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    run(lambda: h.gemm_pp(x, True, w13, True, c, 0.0, 1), f"w13 fwd (K-major x K-major) {T} x {2 * F} x {d}")
    cs = torch.empty(8192, 8192, device="cuda", dtype=torch.bfloat16)
    run(lambda: h.gemm_pp(xs, True, ws, True, cs, 0.0, 1), "square 8192^3 (K-major x K-major)")


if __name__ == "__main__":
    main()
