"""Offline GPT-2 BPE oracle (stands in for ``tiktoken.get_encoding("gpt2")``, which
is not installable here).

Pure Python, deliberately naive and independent of the C++ core: the GPT-2
regex from the ``regex`` module, then for each pre-token repeatedly merge the
adjacent pair with the lowest merge rank (leftmost on ties) -- the algorithm
tiktoken implements -- over the fixture files ``gpt2_vocab.json`` /
``gpt2_merges.txt``.  Special tokens listed in ``allowed_special`` are split
out longest-first and mapped to their ids.
"""

from __future__ import annotations

import json
from functools import lru_cache
from pathlib import Path

import regex

FIXTURES = Path(__file__).resolve().parent / "fixtures"
PAT = regex.compile(r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")


@lru_cache
def _byte_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


class GPT2Oracle:
    def __init__(self, vocab_path=FIXTURES / "gpt2_vocab.json", merges_path=FIXTURES / "gpt2_merges.txt"):
        dec = {v: k for k, v in _byte_unicode().items()}
        raw = json.loads(Path(vocab_path).read_text(encoding="utf-8"))
        self.encoder = {bytes(dec[c] for c in tok): i for tok, i in raw.items()}
        self.decoder = {i: b for b, i in self.encoder.items()}
        self.ranks = {}
        with open(merges_path, encoding="utf-8") as f:
            for line in f:
                parts = line.rstrip().split(" ")
                if len(parts) == 2 and not line.startswith("#version"):
                    pair = (bytes(dec[c] for c in parts[0]), bytes(dec[c] for c in parts[1]))
                    self.ranks.setdefault(pair, len(self.ranks))
        self.special = {"<|endoftext|>": 50256}

    def _bpe(self, word: bytes) -> list[int]:
        parts = [bytes([b]) for b in word]
        while len(parts) > 1:
            best, best_i = None, -1
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best is None or r < best):
                    best, best_i = r, i
            if best is None:
                break
            parts = parts[:best_i] + [parts[best_i] + parts[best_i + 1]] + parts[best_i + 2 :]
        return [self.encoder[p] for p in parts]

    def _encode_ordinary(self, text: str) -> list[int]:
        out = []
        for m in PAT.finditer(text):
            out.extend(self._bpe(m.group().encode("utf-8")))
        return out

    def encode(self, text: str, allowed_special: set[str] | None = None) -> list[int]:
        specials = sorted(allowed_special or (), key=len, reverse=True)
        if not specials:
            return self._encode_ordinary(text)
        rx = "(" + "|".join(regex.escape(s) for s in specials) + ")"
        out: list[int] = []
        for part in regex.split(rx, text):
            if part in self.special and part in specials:
                out.append(self.special[part])
            elif part:
                out.extend(self._encode_ordinary(part))
        return out

    def decode(self, ids: list[int]) -> str:
        inv = {v: k.encode() for k, v in self.special.items()}
        return b"".join(self.decoder.get(i, inv.get(i, b"")) for i in ids).decode("utf-8", errors="replace")
