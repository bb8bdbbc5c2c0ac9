"""Flag `s_waitcnt vmcnt(0)` (full drains of the vector-memory counter) inside loops of MFMA kernels.

A drain inside a tile loop usually means hipcc's wait-count pass could not prove that a register loaded before
the loop (pinned operands behind a branch, a conditional load on the back edge) is complete, and waits for
EVERY outstanding load -- including the next tile's prefetch -- at its first use in every iteration.
usage: python tools/isa_waitcheck.py [csrc/*.hip ...]   (compiles each with hipcc -S for gfx950)"""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "bpe_transformer" / "ops" / "csrc"


def check(src: Path) -> list[str]:
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", str(CSRC), "-S",
                          "--cuda-device-only", str(src), "-o", "-"], capture_output=True, text=True).stdout
    rep = []
    for m in re.finditer(r"^(_Z\w+):\s*$", out, re.M):
        name = m.group(1)
        end = out.find(".Lfunc_end", m.end())
        body = out[m.end():end].split("\n")
        if not any("v_mfma" in t for t in body):
            continue
        depth, n_bad = 0, 0
        for i, t in enumerate(body):
            if "Loop Header" in t:
                depth = 1
            if depth and re.search(r"s_waitcnt\s+vmcnt\(0\)", t):
                nxt = " ".join(x.strip() for x in body[i + 1:i + 3])
                if "v_mfma" in nxt or "ds_read" in nxt:
                    n_bad += 1
        if n_bad:
            rep.append(f"{src.name}: {name[:90]}  in-loop vmcnt(0) before MFMA/LDS read: {n_bad}")
    return rep


if __name__ == "__main__":
    files = [Path(f) for f in sys.argv[1:]] or sorted(CSRC.glob("*.hip"))
    for f in files:
        for line in check(f):
            print(line)
