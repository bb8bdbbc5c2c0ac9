"""Summaries of rocprofv3 hardware-counter runs (``--pmc``), per kernel, with derived rates.

Collect in passes of at most 8 counters, with ``--kernel-trace`` only: never together with the
sys/runtime/hip/hsa/marker trace domains.  For example::

    cd /tmp && export TMPDIR=/tmp
    rocprofv3 --kernel-trace --output-format csv -d out/p1 -o run \\
        --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \\
              SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- python3 benchmarks/attn_bench.py
    rocprofv3 ... -d out/p2 ... --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA \\
              SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- ...
    python -m bpe_transformer.utils.pmc out/p1 out/p2 --match fa_ gemm

Derived values:

* ``mfma_util``: SQ_VALU_MFMA_BUSY_CYCLES (SIMD-cycles with the matrix core busy) over the SIMD-cycles
  available: GRBM_GUI_ACTIVE / n_xcd (kernel cycles) x CUs x 4 SIMDs.  This needs both counters in
  the same kernel's rows; pass the directories of both runs.
* ``valu_per_mfma``, ``lds_per_mfma``: instruction ratios.
* ``lds_conflict``: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
* ``wait_frac``: SQ_WAIT_ANY / SQ_WAVE_CYCLES.
* ``hbm_rd_TBps`` / ``hbm_wr_TBps``: FETCH_SIZE / WRITE_SIZE (KiB) over the kernel's mean duration from the
  same directories' ``*kernel_trace.csv``.  FETCH_SIZE is doubled: on gfx950 it reports exactly half the bytes
  of wide coalesced streaming reads (``MI355X_MICROARCH.md``, FETCH_SIZE note).
"""

from __future__ import annotations

import argparse
import csv
import re
import shutil
import subprocess
from collections import defaultdict
from pathlib import Path

MI355X_CUS = 256
MI355X_XCDS = 8


def short_name(name: str) -> str:
    if name.startswith("_Z") and shutil.which("c++filt"):
        name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*", "", name)[:80]  # drop the parameter list


def load(dirs: list[str | Path], match: list[str] | None = None) -> dict[str, dict[str, float]]:
    """Mean counter value per (kernel, counter) over all dispatches in the given run directories."""
    acc: dict[str, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in Path(d).glob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"]
                if match and not any(m in n for m in match):
                    continue
                acc[short_name(n)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def load_durations(dirs: list[str | Path], match: list[str] | None = None) -> dict[str, float]:
    """Mean dispatch duration (ns) per kernel from the runs' kernel traces."""
    acc: dict[str, list[float]] = defaultdict(list)
    for d in dirs:
        for f in Path(d).glob("*kernel_trace.csv"):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"]
                if match and not any(m in n for m in match):
                    continue
                acc[short_name(n)].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def derive(c: dict[str, float], cus: int = MI355X_CUS, xcds: int = MI355X_XCDS,
           dur_ns: float | None = None) -> dict[str, float]:
    out: dict[str, float] = {}
    g = lambda k: c.get(k)  # noqa: E731
    if dur_ns:
        out["dur_us"] = dur_ns / 1e3
        if g("FETCH_SIZE") is not None:
            out["hbm_rd_TBps"] = 2 * g("FETCH_SIZE") * 1024 / dur_ns / 1e3
        if g("WRITE_SIZE") is not None:
            out["hbm_wr_TBps"] = g("WRITE_SIZE") * 1024 / dur_ns / 1e3
    if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
        out["mfma_util"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / (g("GRBM_GUI_ACTIVE") / xcds * cus * 4)
    if g("SQ_INSTS_MFMA"):
        if g("SQ_INSTS_VALU") is not None:
            out["valu_per_mfma"] = g("SQ_INSTS_VALU") / g("SQ_INSTS_MFMA")
        if g("SQ_INSTS_LDS") is not None:
            out["lds_per_mfma"] = g("SQ_INSTS_LDS") / g("SQ_INSTS_MFMA")
    if g("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict"] = (g("SQ_LDS_BANK_CONFLICT") or 0.0) / g("SQ_LDS_IDX_ACTIVE")
    if g("SQ_WAVE_CYCLES"):
        if g("SQ_WAIT_ANY") is not None:
            out["wait_frac"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
        if g("SQ_ACTIVE_INST_ANY") is not None:
            out["issue_frac"] = g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES")
    return out


def report(dirs: list[str | Path], match: list[str] | None = None) -> str:
    data = load(dirs, match)
    durs = load_durations(dirs, match)
    lines = []
    for k in sorted(data):
        d = derive(data[k], dur_ns=durs.get(k))
        lines.append(f"## {k}")
        if d:
            lines.append("derived: " + ", ".join(f"{n}={v:.3g}" for n, v in d.items()))
        lines += [f"    {c:28s} {v:.4g}" for c, v in sorted(data[k].items())]
        lines.append("")
    return "\n".join(lines)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", nargs="*", default=None, help="substrings of kernel names to keep")
    a = ap.parse_args()
    print(report(a.dirs, a.match))


if __name__ == "__main__":
    main()
