"""Import of the C++ tokenizer core, building it in-tree on first use if needed."""

from __future__ import annotations

import importlib

try:
    from . import _bpe_native as native  # noqa: F401
except ImportError:  # not built yet: compile (g++, seconds) and import
    from ._native_build import build

    build()
    native = importlib.import_module("bpe_transformer.tokenization._bpe_native")
