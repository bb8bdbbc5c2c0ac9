"""Import of the C++ tokenizer core, building it in-tree on first use if needed."""

from __future__ import annotations

import importlib

from ._native_build import build, is_fresh

if not is_fresh():  # not built, or built from other sources (content stamp): compile (g++, seconds) first
    build()
native = importlib.import_module("bpe_transformer.tokenization._bpe_native")
