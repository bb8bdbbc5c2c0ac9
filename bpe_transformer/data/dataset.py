"""Token datasets: memory-mapped token files and synthetic token streams.

Token files are flat little-endian arrays (``uint16`` when the vocabulary fits,
else ``uint32``) so that a multi-GB corpus is ``np.memmap``-ed, never loaded:
the batch sampler gathers only the windows it needs.
"""

from __future__ import annotations

from collections.abc import Iterable
from pathlib import Path

import numpy as np


def token_dtype(vocab_size: int) -> np.dtype:
    return np.dtype(np.uint16) if vocab_size <= 65536 else np.dtype(np.uint32)


def write_tokens(ids: Iterable[int], path: str | Path, vocab_size: int = 65536, chunk: int = 1 << 20) -> int:
    """Stream token ids to a flat binary file; returns the number of tokens written."""
    dt = token_dtype(vocab_size)
    n = 0
    buf: list[int] = []
    with open(path, "wb") as f:
        for t in ids:
            buf.append(t)
            if len(buf) >= chunk:
                np.asarray(buf, dtype=dt).tofile(f)
                n += len(buf)
                buf.clear()
        if buf:
            np.asarray(buf, dtype=dt).tofile(f)
            n += len(buf)
    return n


def load_tokens(path: str | Path, vocab_size: int = 65536) -> np.memmap:
    """Memory-map a token file written by :func:`write_tokens` (or any flat uint16/uint32 array)."""
    return np.memmap(path, dtype=token_dtype(vocab_size), mode="r")


def synthetic_tokens(vocab_size: int, n_tokens: int, seed: int = 0) -> np.ndarray:
    """Uniform random token stream (benchmarks: 'synthetic data of the named shape')."""
    rng = np.random.default_rng(seed)
    return rng.integers(0, vocab_size, size=n_tokens, dtype=np.int64).astype(token_dtype(vocab_size))
