"""Data pipeline: batch sampling, memmapped token files, synthetic tokens."""

from .batch import BatchLoader, get_batch
from .dataset import load_tokens, synthetic_tokens, token_dtype, write_tokens

__all__ = ["BatchLoader", "get_batch", "load_tokens", "synthetic_tokens", "token_dtype", "write_tokens"]
