"""Positional embeddings (the reference's ``embeddings/`` package; its ``rope.py`` is empty)."""

from .rope import RotaryPositionalEmbedding, apply_rope

__all__ = ["RotaryPositionalEmbedding", "apply_rope"]
