"""Byte-level BPE trainer (reference: ``bpe_transformer/tokenization/bpe_trainer.py``).

Same public surface as the reference ``BPETrainer`` (class :10):
``BPETrainer(vocab_size, special_tokens)`` (:69), ``.train(input_path, n_workers)``
(:141), ``.vocab`` / ``.merges`` / ``.special_tokens`` / ``.vocab_size`` (:95-113),
``.add_new_vocab`` (:131), ``.save_trainer(output_dir)`` (:447).

Differences by design:
  * canonical BPE counts (the reference double-counts self-pairs);
  * special tokens get ids 256.. in LIST order (the reference numbers them from
    a ``set``, i.e. nondeterministically);
  * the counting + merge loop is the threaded C++ core (``_bpe_native``).
Ids: 0..255 are the single bytes, then the specials, then merges in order.
Ties between equally frequent pairs go to the lexicographically greater
``(bytes, bytes)`` pair, as in the reference (:59-64).
"""

from __future__ import annotations

from multiprocessing import cpu_count
from pathlib import Path

from ..settings import DEFAULT_OUTPUT_DIR
from ._native import native
from .serialization import save_merges, save_vocab


class BPETrainer:
    def __init__(self, vocab_size: int, special_tokens: list[str] | None = None):
        specials: list[str] = []
        for s in special_tokens or []:
            if s not in specials:
                specials.append(s)
        if vocab_size < 256 + len(specials):
            raise ValueError(f"vocab_size {vocab_size} < 256 byte tokens + {len(specials)} special tokens")
        self._vocab_size = vocab_size
        self._special_tokens = specials
        self._vocab: dict[int, bytes] = self._build_initial_vocab()
        self._merges: list[tuple[bytes, bytes]] = []

    @property
    def vocab(self) -> dict[int, bytes]:
        return self._vocab

    @property
    def merges(self) -> list[tuple[bytes, bytes]]:
        return self._merges

    @property
    def special_tokens(self) -> list[str]:
        return list(self._special_tokens)

    @property
    def vocab_size(self) -> int:
        return self._vocab_size

    def _build_initial_vocab(self) -> dict[int, bytes]:
        vocab = {i: bytes([i]) for i in range(256)}
        for j, s in enumerate(self._special_tokens):
            vocab[256 + j] = s.encode("utf-8")
        return vocab

    def add_new_vocab(self, id: int, new_value: bytes) -> None:  # noqa: A002 (reference name)
        if id in self._vocab:
            raise ValueError(f"id {id} already in vocab")
        self._vocab[id] = new_value

    def train(self, input_path: Path | str, n_workers: int | None = None) -> None:
        """Pre-tokenise ``input_path`` (threads) and learn merges until ``vocab_size`` (or no pairs left)."""
        n = n_workers if n_workers and n_workers > 0 else cpu_count()
        vocab, merges = native.train_file(str(input_path), self._vocab_size, self._special_tokens, int(n))
        self._vocab = vocab
        self._merges = merges

    def train_from_counts(self, counts: dict[bytes, int]) -> None:
        """Learn merges from an explicit ``{pretoken_bytes: count}`` table."""
        self._vocab, self._merges = native.train_from_counts(counts, self._vocab_size, self._special_tokens)

    def save_trainer(self, output_dir: Path | str = DEFAULT_OUTPUT_DIR / "tokenizer" / "bpe_trainer") -> None:
        """Write ``vocab.pkl`` and ``merges.pkl`` (pickle protocol 4, reference-compatible)."""
        out = Path(output_dir)
        out.mkdir(parents=True, exist_ok=True)
        save_vocab(self._vocab, out / "vocab.pkl")
        save_merges(self._merges, out / "merges.pkl")
