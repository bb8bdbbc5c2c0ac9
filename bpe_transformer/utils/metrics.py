"""Metrics logging and step timing.

``MetricsLogger`` writes one JSON object per line (loss, lr, grad-norm,
tokens/s, MFU, memory) and mirrors a short line to ``logging``.
``StepTimer`` brackets regions with device events (``hipEvent`` under ROCm) so
timing never forces a host sync inside the step; ``summary()`` syncs once.
"""

from __future__ import annotations

import json
import logging
import time
from collections import defaultdict
from pathlib import Path

import torch

log = logging.getLogger("bpe_transformer")


def setup_logging(rank: int = 0, level: int = logging.INFO) -> None:
    fmt = f"[%(asctime)s r{rank}] %(message)s"
    logging.basicConfig(level=level if rank == 0 else logging.WARNING, format=fmt, datefmt="%H:%M:%S")


class MetricsLogger:
    def __init__(self, path: str | Path | None = None, rank: int = 0):
        self.rank = rank
        self.path = Path(path) if path else None
        self._f = None
        if self.path is not None and rank == 0:
            self.path.parent.mkdir(parents=True, exist_ok=True)
            self._f = open(self.path, "a")

    def log(self, **fields) -> None:
        if self.rank != 0:
            return
        fields.setdefault("time", time.time())
        if self._f is not None:
            self._f.write(json.dumps(fields) + "\n")
            self._f.flush()
        short = " ".join(f"{k}={v:.4g}" if isinstance(v, float) else f"{k}={v}" for k, v in fields.items()
                         if k != "time")
        log.info(short)

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None


class StepTimer:
    """Accumulates per-region device time with events; no sync until :meth:`summary`."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending: list[tuple[str, torch.cuda.Event, torch.cuda.Event]] = []
        self.totals: dict[str, float] = defaultdict(float)
        self.counts: dict[str, int] = defaultdict(int)

    def region(self, name: str):
        timer = self

        class _R:
            def __enter__(self_inner):
                if timer.enabled:
                    self_inner.s = torch.cuda.Event(enable_timing=True)
                    self_inner.e = torch.cuda.Event(enable_timing=True)
                    self_inner.s.record()
                return self_inner

            def __exit__(self_inner, *exc):
                if timer.enabled:
                    self_inner.e.record()
                    timer._pending.append((name, self_inner.s, self_inner.e))
                return False

        return _R()

    def summary(self) -> dict[str, float]:
        if self._pending:
            torch.cuda.synchronize()
            for name, s, e in self._pending:
                self.totals[name] += s.elapsed_time(e)
                self.counts[name] += 1
            self._pending.clear()
        return {k: self.totals[k] / max(self.counts[k], 1) for k in self.totals}


def device_memory_gb() -> float:
    if not torch.cuda.is_available():
        return 0.0
    return torch.cuda.max_memory_allocated() / 1e9
