#!/usr/bin/env python3
"""Instruction census of the kernels in a hipcc ``-S`` gfx950 assembly file.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S x.hip -o x.s
    python tools/isa_census.py x.s [name-substring] [--top N]

Prints, per kernel whose mangled name contains the substring: instruction count, VGPR / spill counts from
the metadata, and the most frequent opcodes.  Used to check what a source change did to a kernel's body
(e.g. a division that expands to a v_div_scale / v_div_fmas / v_div_fixup sequence, or scratch spills).
"""

from __future__ import annotations

import argparse
import re
from collections import Counter


def kernels(text: str) -> dict[str, list[str]]:
    out: dict[str, list[str]] = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        s = line.strip()
        if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
            continue
        out[cur].append(s.split()[0])
    return out


def metadata(text: str) -> dict[str, dict[str, int]]:
    meta: dict[str, dict[str, int]] = {}
    for block in re.split(r"\n  - ", text):
        m = re.search(r"\.name:\s+(\S+)", block)
        if not m:
            continue
        d = {}
        for key in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "agpr_count"):
            mm = re.search(rf"\.{key}:\s+(\d+)", block)
            if mm:
                d[key] = int(mm.group(1))
        meta[m.group(1)] = d
    return meta


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("substr", nargs="?", default="")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    text = open(a.asm).read()
    meta = metadata(text)
    for name, ops in kernels(text).items():
        if a.substr not in name:
            continue
        c = Counter(ops)
        print(f"{name}  instrs={len(ops)}  {meta.get(name, {})}")
        for op, n in c.most_common(a.top):
            print(f"    {op:32s} {n}")


if __name__ == "__main__":
    main()
