"""MFMA placement check for the barrier-phased kernels (ping-pong GEMM, attention): for every kernel in a
hipcc -S file, the number of MFMAs between consecutive s_barrier instructions, in program order.  A ping-pong
main loop must show its per-phase count in every section (16 bf16 / 8 fp8 for gemm_pp); a section with 2-4x
that next to empty ones means the compiler moved MFMAs across the phase barriers.  Counts are in static
order: a rotated loop shows one section split between the loop top and bottom (e.g. 8 | 16 | 16 | 16 | 8 for
the weight-gradient schedule, 16 per section at run time).

    python tools/isa_mfma_sections.py file.s [kernel_substring]
"""
import re
import sys
from collections import Counter


def sections(body: str) -> list[int]:
    out, n = [], 0
    for ln in body.split("\n"):
        t = ln.strip()
        if t.startswith("v_mfma"):
            n += 1
        elif t.startswith("s_barrier"):
            out.append(n)
            n = 0
    out.append(n)
    return out


def main():
    src = open(sys.argv[1]).read()
    key = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"^(_Z\S+):(?:\s*;.*)?$", src, re.M):
        name = m.group(1)
        if key not in name:
            continue
        end = src.find(".Lfunc_end", m.end())
        sec = sections(src[m.end():end])
        if not any(sec):
            continue
        nz = Counter(x for x in sec if x)
        print(f"{name[:90]}  sections with MFMAs: {dict(sorted(nz.items()))}")


if __name__ == "__main__":
    main()
