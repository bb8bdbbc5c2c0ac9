"""GPT-2 pre-tokenisation: chunking, special-token splitting, counting.

Public API mirrors the reference module
(``bpe_transformer/tokenization/preprocessing/pretokenization.py``):
``pretokenize`` (:41), ``parallel_pretokenization`` (:73),
``find_chunk_boundaries`` (:114), ``pretokenize_chunk`` (:171),
``split_on_special_tokens`` (:211), ``pretokenize_text`` (:238),
``serial_pretokenization`` (:255).  Counters are keyed like the reference's:
``tuple(pretoken_bytes)`` (a tuple of byte values).

Implementation: the regex matcher, the special-token splitter and the
counting loop run in the C++ core (``_bpe_native``) with std::threads instead
of a process pool (no pickling, GIL released).  Chunk boundaries are taken at
special tokens (or, without specials, at positions that provably cannot
change the pre-tokenisation), so counts never depend on the worker count.
"""

from __future__ import annotations

import os
from collections import Counter
from multiprocessing import cpu_count
from pathlib import Path
from typing import BinaryIO

import regex as re

from ...settings import ENCODING_STD
from .._native import native


def _workers(n_workers: int | None) -> int:
    if n_workers is None or n_workers == 0:
        n_workers = 4
    return max(1, min(int(n_workers), cpu_count()))


def _to_counter(d: dict[bytes, int]) -> Counter:
    return Counter({tuple(k): v for k, v in d.items()})


def pretokenize(
    file_path: Path,
    training: bool | None = True,
    parallel_processing: bool | None = True,
    n_workers: int | None = 4,
    special_tokens: list[str] | None = None,
) -> Counter:
    """Count pre-tokens of a file (parallel by default)."""
    if parallel_processing:
        return parallel_pretokenization(file_path, n_workers=n_workers, training=training,
                                        special_tokens=special_tokens)
    return serial_pretokenization(file_path, training=training, special_tokens=special_tokens)


def parallel_pretokenization(file_path: Path, n_workers: int | None = None, training: bool | None = True,
                             special_tokens: list[str] | None = None) -> Counter:
    specials = list(special_tokens or [])
    if training:
        return _to_counter(native.count_pretokens_file(str(file_path), specials, _workers(n_workers)))
    with open(file_path, "rb") as f:
        data = f.read().decode(ENCODING_STD, errors="ignore")
    return _count_text_keep_specials(data, specials)


def serial_pretokenization(file_path: Path, training: bool | None = True,
                           special_tokens: list[str] | None = None) -> Counter:
    specials = list(special_tokens or [])
    if training:
        return _to_counter(native.count_pretokens_file(str(file_path), specials, 1))
    with open(file_path, "rb") as f:
        data = f.read().decode(ENCODING_STD, errors="ignore")
    return _count_text_keep_specials(data, specials)


def _count_text_keep_specials(text: str, specials: list[str]) -> Counter:
    """Encode-mode counting: specials are kept whole as their own pre-tokens."""
    counter: Counter = Counter()
    for part in split_on_special_tokens(text, training=False, special_tokens=specials):
        if not part:
            continue
        if part in specials:
            counter[tuple(part.encode(ENCODING_STD))] += 1
            continue
        for k, v in native.count_pretokens_text(part.encode(ENCODING_STD), [], 1).items():
            counter[tuple(k)] += v
    return counter


def find_chunk_boundaries(file: BinaryIO, desired_num_chunks: int, special_tokens: list[str] | None = None
                          ) -> list[int]:
    """Byte offsets splitting ``file`` into up to ``desired_num_chunks`` pieces, each boundary at the
    earliest special token (or ``b"\\n"`` when there are none) after a uniform guess; deduplicated,
    so fewer chunks may come back (reference :114-168)."""
    split_tokens = [t.encode(ENCODING_STD) for t in special_tokens] if special_tokens else [b"\n"]
    file.seek(0, os.SEEK_END)
    size = file.tell()
    file.seek(0)
    chunk = size // max(desired_num_chunks, 1)
    bounds = [i * chunk for i in range(desired_num_chunks + 1)]
    bounds[-1] = size
    mini = 4096
    maxlen = max(len(t) for t in split_tokens)
    for bi in range(1, len(bounds) - 1):
        pos = bounds[bi]
        while True:
            file.seek(pos)
            buf = file.read(mini + maxlen - 1)
            if not buf:
                bounds[bi] = size
                break
            found = [p for p in (buf.find(t) for t in split_tokens) if p != -1]
            if found:
                bounds[bi] = pos + min(found)
                break
            pos += mini
    return sorted(set(bounds))


def pretokenize_chunk(file_path: Path, start: int, end: int, training: bool | None = True,
                      special_tokens: list[str] | None = None) -> Counter:
    with open(file_path, "rb") as f:
        f.seek(start)
        data = f.read(end - start)
    specials = list(special_tokens or [])
    if training:
        return _to_counter(native.count_pretokens_text(native.sanitize_utf8(data), specials, 1))
    return _count_text_keep_specials(data.decode(ENCODING_STD, errors="ignore"), specials)


def split_on_special_tokens(text: str, training: bool | None = True, special_tokens: list[str] | None = None
                            ) -> list[str]:
    """Split ``text`` on special tokens, longest first; training drops them, encode mode keeps them."""
    if not special_tokens:
        return [text]
    escaped = [re.escape(t) for t in sorted(special_tokens, key=len, reverse=True)]
    pattern = "|".join(escaped) if training else f"({'|'.join(escaped)})"
    return re.split(pattern, text)


def pretokenize_text(text: str) -> list[bytes]:
    """GPT-2 regex pre-tokens of ``text`` as utf-8 bytes (C++ matcher)."""
    return native.pretokenize(text.encode(ENCODING_STD))
