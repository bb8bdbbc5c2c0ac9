"""Tokenizer artifact I/O.

Byte-compatible with the reference (``bpe_trainer.py:447-472``,
``bpe_tokenizer.py:292-337``): ``vocab.pkl`` is a pickled
``dict[int, bytes]`` and ``merges.pkl`` a pickled ``list[tuple[bytes, bytes]]``
(protocol 4).  Loading never runs an unpickler: :mod:`.safe_pickle` interprets
the opcode stream itself and accepts only builtin data (ints, bytes, lists,
tuples, dicts), so a tampered file cannot execute code -- these two artifacts
only ever contain builtin containers, ints and bytes.

Also reads/writes the GPT-2 text formats (``vocab.json`` + ``merges.txt`` with
the byte-to-unicode remapping).
"""

from __future__ import annotations

import json
import pickle
from functools import lru_cache
from pathlib import Path

from . import safe_pickle

PICKLE_PROTOCOL = 4


def safe_pickle_load(path: str | Path):
    """Builtin data from a pickle file, without unpickling (:func:`.safe_pickle.load`)."""
    return safe_pickle.load(path)


def save_vocab(vocab: dict[int, bytes], path: str | Path) -> None:
    with open(path, "wb") as f:
        pickle.dump(vocab, f, protocol=PICKLE_PROTOCOL)


def save_merges(merges: list[tuple[bytes, bytes]], path: str | Path) -> None:
    with open(path, "wb") as f:
        pickle.dump(merges, f, protocol=PICKLE_PROTOCOL)


def load_vocab(path: str | Path) -> dict[int, bytes]:
    v = safe_pickle_load(path)
    if not isinstance(v, dict) or not all(isinstance(k, int) and isinstance(b, bytes) for k, b in v.items()):
        raise ValueError(f"{path}: not a dict[int, bytes] vocab")
    return v


def load_merges(path: str | Path) -> list[tuple[bytes, bytes]]:
    m = safe_pickle_load(path)
    if not isinstance(m, list) or not all(isinstance(t, tuple) and len(t) == 2 for t in m):
        raise ValueError(f"{path}: not a list[tuple[bytes, bytes]] merges list")
    return [(bytes(a), bytes(b)) for a, b in m]


@lru_cache
def gpt2_bytes_to_unicode() -> dict[int, str]:
    """GPT-2's reversible byte -> printable-unicode map."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


def load_gpt2_files(vocab_json: str | Path, merges_txt: str | Path, special_tokens: list[str] | None = None):
    """Read GPT-2 style ``vocab.json``/``merges.txt`` into (vocab dict[int, bytes], merges)."""
    dec = {v: k for k, v in gpt2_bytes_to_unicode().items()}
    with open(vocab_json, encoding="utf-8") as f:
        raw = json.load(f)
    vocab = {int(i): bytes(dec[c] for c in tok) for tok, i in raw.items()}
    merges = []
    with open(merges_txt, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip().split(" ")
            if len(parts) == 2 and not line.startswith("#version"):
                merges.append((bytes(dec[c] for c in parts[0]), bytes(dec[c] for c in parts[1])))
    if special_tokens:
        have = set(vocab.values())
        for s in special_tokens:
            b = s.encode("utf-8")
            if b not in have:
                vocab[len(vocab)] = b
    return vocab, merges


def save_gpt2_files(vocab: dict[int, bytes], merges: list[tuple[bytes, bytes]], vocab_json: str | Path,
                    merges_txt: str | Path) -> None:
    enc = gpt2_bytes_to_unicode()
    with open(vocab_json, "w", encoding="utf-8") as f:
        json.dump({"".join(enc[b] for b in tok): i for i, tok in vocab.items()}, f, ensure_ascii=False)
    with open(merges_txt, "w", encoding="utf-8") as f:
        for a, b in merges:
            f.write("".join(enc[x] for x in a) + " " + "".join(enc[x] for x in b) + "\n")
