"""``train_bpe`` entry point (reference: ``bpe_transformer/main.py:8-17``)."""

from __future__ import annotations

from multiprocessing import cpu_count
from pathlib import Path

from .tokenization.bpe_trainer import BPETrainer

N_WORKERS = cpu_count()


def train_bpe(input_path: str | Path, vocab_size: int, special_tokens: list[str] | None = None,
              n_workers: int | None = None) -> tuple[dict[int, bytes], list[tuple[bytes, bytes]]]:
    """Train a byte-level BPE tokenizer on ``input_path``; returns ``(vocab, merges)``.

    ``vocab_size`` must be at least 256 + len(special_tokens) (the reference's
    check was off by one).
    """
    specials = list(dict.fromkeys(special_tokens or []))
    if vocab_size < 256 + len(specials):
        raise ValueError("Input vocab_size is invalid: value too small.")
    bpe = BPETrainer(vocab_size=vocab_size, special_tokens=specials)
    bpe.train(input_path=input_path, n_workers=n_workers or N_WORKERS)
    return bpe.vocab, bpe.merges
