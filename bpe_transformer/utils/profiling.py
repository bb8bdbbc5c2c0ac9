"""Profiling helpers.

* :func:`torch_profile` -- a ``torch.profiler`` context with HIP activities and
  a wait/warmup/active schedule, exporting a Chrome trace + a kernel table.
* :func:`summarize_rocprof_stats` -- turns a ``rocprofv3 --kernel-trace --stats``
  ``*_kernel_stats.csv`` into a per-kernel table grouped by component
  (GEMM / attention / norm / loss / optimizer / elementwise), the form the
  ``profiles/`` summaries are committed in.
* :func:`mfu` -- model FLOPs utilisation against the dense bf16 MFMA peak
  (2.5 PF/s per MI355X; never the 2:1-sparsity headline number).
"""

from __future__ import annotations

import csv
from collections import defaultdict
from contextlib import contextmanager
from pathlib import Path

import torch

MI355X_BF16_DENSE_FLOPS = 2.5e15
MI355X_FP8_DENSE_FLOPS = 5.0e15

_GROUPS = [
    ("attention", ("fa_fwd", "fa_bwd", "fa_dq", "flash")),
    ("gemm", ("Cijk_", "gemm", "Gemm", "_MT")),
    ("rmsnorm", ("rmsnorm", "colsum")),
    ("swiglu/act", ("swiglu", "act_fwd", "act_bwd")),
    ("cross_entropy", ("ce_fwd", "softmax")),
    ("optimizer", ("adamw", "sumsq", "norm_finalize", "scale_kernel")),
    ("embedding", ("embed_",)),
    ("fp8 quant", ("cast_fp8", "update_scales")),
    ("rope", ("rope_kernel",)),
    ("comm", ("nccl", "rccl", "Reduce", "AllReduce")),
]


def classify_kernel(name: str) -> str:
    for g, keys in _GROUPS:
        if any(k in name for k in keys):
            return g
    return "elementwise/other"


def _load_stats(path: str | Path) -> list[dict]:
    """Per-kernel rows from a ``*_kernel_stats.csv`` or a rocpd SQLite ``*_results.db`` (rocprofv3's
    default output format on ROCm 7)."""
    path = Path(path)
    if path.suffix != ".db":
        return list(csv.DictReader(open(path)))
    import sqlite3

    con = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
    try:
        q = "select name, count(*), sum(duration), avg(duration) from kernels group by name"  # ns
        rows = [{"Name": n, "Calls": c, "TotalDurationNs": t, "AverageNs": a} for n, c, t, a in con.execute(q)]
    finally:
        con.close()
    tot = sum(r["TotalDurationNs"] for r in rows) or 1
    for r in rows:
        r["Percentage"] = 100.0 * r["TotalDurationNs"] / tot
    return rows


def summarize_rocprof_stats(csv_path: str | Path, steps: int | None = None) -> str:
    rows = _load_stats(csv_path)
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    groups: dict[str, float] = defaultdict(float)
    for r in rows:
        groups[classify_kernel(r["Name"])] += float(r["TotalDurationNs"])
    per = f" (per step: /{steps})" if steps else ""
    lines = [f"total kernel time {tot / 1e6:.2f} ms{per}", "", "| component | ms | % |", "|---|---|---|"]
    for g, v in sorted(groups.items(), key=lambda kv: -kv[1]):
        ms = v / 1e6 / (steps or 1)
        lines.append(f"| {g} | {ms:.3f} | {100 * v / tot:.1f} |")
    lines += ["", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    return "\n".join(lines)


def mfu(tokens_per_s: float, flops_per_token: float, n_gpus: int = 1, peak: float = MI355X_BF16_DENSE_FLOPS) -> float:
    return tokens_per_s * flops_per_token / (peak * n_gpus)


@contextmanager
def torch_profile(out_dir: str | Path, wait: int = 1, warmup: int = 1, active: int = 3):
    from torch.profiler import ProfilerActivity, profile, schedule

    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])

    def _ready(p):
        p.export_chrome_trace(str(out / f"trace_{p.step_num}.json"))
        (out / "kernels.txt").write_text(p.key_averages().table(sort_by="cuda_time_total", row_limit=60))

    with profile(activities=acts, schedule=schedule(wait=wait, warmup=warmup, active=active),
                 on_trace_ready=_ready, record_shapes=False) as prof:
        yield prof


if __name__ == "__main__":
    import sys

    print(summarize_rocprof_stats(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None))
