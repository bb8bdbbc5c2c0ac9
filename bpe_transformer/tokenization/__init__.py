"""Byte-level BPE tokenizer: trainer, encoder/decoder, pre-tokenisation (C++ core)."""

from .bpe_tokenizer import BPETokenizer
from .bpe_trainer import BPETrainer
from .tokenizer import Tokenizer

__all__ = ["BPETokenizer", "BPETrainer", "Tokenizer"]
