"""Summarise a rocprofv3 ``--kernel-trace`` CSV into the markdown tables under ``profiles/``.

usage: python tools/prof_summary.py <kernel_trace.csv | results.db> --steps 5 --warmup 3 [--title T] [--note N]

Takes either the CSV (``--output-format csv``) or the rocpd SQLite database that
rocprofv3 writes by default on ROCm 7.x (``kernels`` view).

Only the timed steps count: the trace is cut at the ``(warmup+1)``-th launch of
the embedding forward kernel (one per step), so warmup launches, TunableOp
lookups and init kernels are excluded.  Times are per step.  Kernels are bucketed
into components by name so the split matches docs/performance.md.
"""

from __future__ import annotations

import argparse
import csv
from collections import defaultdict

_COMPONENTS = [
    ("gemm", ("Cijk", "gemm")),  # library (Tensile/hipBLASLt) names first: they contain arbitrary tags
    ("comm", ("nccl", "rccl", "allreduce", "AllReduce")),
    ("optimizer", ("adamw", "adam", "l2norm", "grad_norm", "clip")),
    ("attention", ("fa_", "flash", "attn", "rope")),
    ("cross_entropy", ("ce_fwd", "ce_bwd", "cross_entropy", "xent")),
    ("rmsnorm", ("rmsnorm", "norm_")),
    ("swiglu/act", ("swiglu", "silu", "gelu")),
    ("embedding", ("embed",)),
    ("gemm", ("MT256", "MT128", "MT64", "fp8_", "gemv")),
]


def component(name: str) -> str:
    low = name.lower()
    for comp, keys in _COMPONENTS:
        if any(k.lower() in low for k in keys):
            return comp
    return "elementwise/other"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--marker", default="embed_fwd", help="kernel launched once per step")
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    ap.add_argument("--note", default="")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()

    rows = []
    if a.csv.endswith(".db"):
        import sqlite3

        con = sqlite3.connect(a.csv)
        rows = [(int(b), int(e), n) for b, e, n in con.execute("select start, end, name from kernels")]
        con.close()
    else:
        with open(a.csv) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, (_, _, n) in enumerate(rows) if a.marker in n]
    if len(marks) < a.warmup + 1:
        raise SystemExit(f"only {len(marks)} '{a.marker}' launches; cannot skip {a.warmup} warmup steps")
    timed = rows[marks[a.warmup]:]
    s = a.steps
    wall = (max(e for _, e, _ in timed) - timed[0][0]) / 1e6 / s
    per_k: dict[str, list[float]] = defaultdict(list)
    for b, e, n in timed:
        per_k[n].append((e - b) / 1e6)
    busy = sum(sum(v) for v in per_k.values()) / s
    per_c: dict[str, float] = defaultdict(float)
    for n, v in per_k.items():
        per_c[component(n)] += sum(v) / s

    out = [f"# {a.title}", ""]
    if a.note:
        out += [a.note, ""]
    out += [f"wall span {wall:.2f} ms/step, kernel busy {busy:.2f} ms/step ({100 * busy / wall:.1f} %)", ""]
    out += ["| component | ms/step | % |", "|---|---|---|"]
    for c, t in sorted(per_c.items(), key=lambda x: -x[1]):
        out.append(f"| {c} | {t:.3f} | {100 * t / busy:.1f} |")
    out += ["", "| kernel | calls/step | ms/step | avg us | % |", "|---|---|---|---|---|"]
    for n, v in sorted(per_k.items(), key=lambda x: -sum(x[1]))[: a.top]:
        t = sum(v) / s
        out.append(f"| `{n[:90]}` | {len(v) / s:.1f} | {t:.3f} | {1e3 * sum(v) / len(v):.1f} | {100 * t / busy:.2f} |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
